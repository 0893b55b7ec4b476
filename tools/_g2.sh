mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -q -x -m gpu > gpurun_out/t.log 2>&1; tail -n 3 gpurun_out/t.log
for m in mfcc_bgru spec_bgru fbanks_cnn; do
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 3 --no-cpu-baseline --no-feature-roofline 2>/dev/null | tail -n 1 > gpurun_out/b_$m.json || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_$m.json'));print('$m',d['value'],d['ms_per_step'],{k:round(v['ms_total']/d['steps'],3) for k,v in d['kernels'].items()})"
done
