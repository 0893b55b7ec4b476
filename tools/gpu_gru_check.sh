#!/bin/bash
# A recurrence change on the GPU:  gpurun --timeout 900 -- bash tools/gpu_gru_check.sh TAG ["-k expression"] [A/B srk options]
# the 16-bit GRU tests, then bench lines (graph replays) of cfg2 (fp32 + the bf16 record) and cfg5 (fp16), each at
# the default options and, with a third argument, again under SRK_OPTIONS=<it>.
set -o pipefail
TAG=${1:-gru}
KEXPR=${2:-gru}
AB=${3:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lowprec_gpu.py tests/test_trainstep_lowprec_gpu.py -k "$KEXPR" -x -v \
  --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || exit $rc
line() {   # line NAME ARGS...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs --no-feature-roofline --no-h2d "$@" \
    > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || return $?
  python3 -c "
import json
d = json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1])
b = d.get('bf16') or {}
print('$name', d['dtype'], d['value'], d['ms_per_step'], '| bf16', b.get('value'), b.get('ms_per_step'))
k = d.get('kernels', {})
print('   ', {n: v['ms_total'] for n, v in k.items() if n.startswith('gru')})
"
}
line cfg2 --steps 30 && line cfg5 --model spec_bgru --precision fp16 --steps 30 || exit $?
if [ -n "$AB" ]; then
  SRK_OPTIONS="$AB" line cfg2_ab --steps 30 && SRK_OPTIONS="$AB" line cfg5_ab --model spec_bgru --precision fp16 --steps 30
fi
