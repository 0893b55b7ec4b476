set -o pipefail
mkdir -p gpurun_out/g15
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g15/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/g15/pytest.log; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert|^E ' gpurun_out/g15/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-feature-roofline > gpurun_out/g15/bench.json 2> gpurun_out/g15/bench.err && python -c "import json;d=json.load(open('gpurun_out/g15/bench.json'));b=d['bf16'];print('mfcc fp32',d['value'],d['ms_per_step'],{k:v['ms_total'] for k,v in d['kernels'].items()},'bf16',b['value'],b['ms_per_step'],{k:v['ms_total'] for k,v in b['kernels'].items()})"
timeout -k 10 120 python tools/gru_trace.py 2>/dev/null | tail -1
