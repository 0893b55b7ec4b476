set -o pipefail
O=gpurun_out/v3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert|^E ' $O/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-feature-roofline > $O/bench$i.json 2> $O/bench$i.err || exit 1
  python -c "import json;d=json.load(open('$O/bench$i.json'));b=d['bf16'];print('fp32',d['value'],'bf16',b['value'],b['ms_per_step'],{k:v['ms_total'] for k,v in b['kernels'].items()})"
done
