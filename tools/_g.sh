set -o pipefail
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_lowprec_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g8/pytest_lp.log 2>&1
rc=$?; tail -2 gpurun_out/g8/pytest_lp.log; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert|^E ' gpurun_out/g8/pytest_lp.log | head -30; exit $rc; }
for m in fbanks_cnn resnet_bgru; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --no-cpu-baseline --no-feature-roofline > gpurun_out/g8/bench_$m.json 2> gpurun_out/g8/bench_$m.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/g8/bench_$m.json'));b=d['bf16'];print('$m fp32',d['value'],d['ms_per_step'],'bf16',b['value'],b['ms_per_step'],{k:v['ms_total'] for k,v in b['kernels'].items()})"
done
