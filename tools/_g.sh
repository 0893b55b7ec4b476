set -o pipefail
mkdir -p gpurun_out/g7
export TMPDIR=/tmp
for m in fbanks_cnn resnet_bgru spec_bgru mfrn_bgru; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --no-cpu-baseline --no-feature-roofline > gpurun_out/g7/bench_$m.json 2> gpurun_out/g7/bench_$m.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/g7/bench_$m.json'));b=d['bf16'];print('$m fp32',d['value'],d['ms_per_step'],'bf16',b['value'],b['ms_per_step'],{k:v['ms_total'] for k,v in b['kernels'].items()})"
done
timeout -k 10 300 python bench.py --model spec_bgru --precision fp16 --steps 10 --no-cpu-baseline --no-feature-roofline > gpurun_out/g7/bench_spec_fp16.json 2> gpurun_out/g7/bench_spec_fp16.err && python -c "import json;d=json.load(open('gpurun_out/g7/bench_spec_fp16.json'));print('spec fp16',d['value'],d['ms_per_step'],d['final_loss'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-feature-roofline > gpurun_out/g7/bench.json 2> gpurun_out/g7/bench.err && python -c "import json;d=json.load(open('gpurun_out/g7/bench.json'));b=d['bf16'];print('mfcc fp32',d['value'],'bf16',b['value'],b['ms_per_step'],{k:v['ms_total'] for k,v in b['kernels'].items()})"
