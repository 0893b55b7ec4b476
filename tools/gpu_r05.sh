#!/bin/bash
# Round-5 GPU call: selected GPU tests, then selected bench commands, each step under its own limit.
#   gpurun --timeout 900 -- bash tools/gpu_r05.sh TAG "tests/a.py tests/b.py" "BENCHARGS1" "BENCHARGS2" ...
# An empty test list skips pytest; every bench command writes $OUT/bench_<i>.json.
set -o pipefail
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?
  tail -1 "$OUT/pytest.log"
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|^E " "$OUT/pytest.log" | head -40; exit $rc; fi
fi
i=0
for args in "$@"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || { echo "bench $i failed"; tail -20 "$OUT/bench_$i.err"; exit 1; }
  python - "$OUT/bench_$i.json" "$args" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
line = "%s: %s %s ms/step %s" % (sys.argv[2], r["value"], r["unit"], r["ms_per_step"])
if "bf16" in r: line += " | bf16 %s (%s ms)" % (r["bf16"]["value"], r["bf16"]["ms_per_step"])
if "h2d" in r: line += " | h2d fp32 %s bf16 %s" % (r["h2d"]["fp32"]["value"], r["h2d"]["bf16"]["value"])
for c in r.get("configs", []): line += " | %s %s %s" % (c["config"], c["dtype"], c["value"])
print(line)
PY
done
if [ -n "$HANDOFF" ]; then
  timeout -k 10 120 tools/_exp/handoff_micro > "$OUT/handoff_micro.txt" 2>&1; rc=$?
  cat "$OUT/handoff_micro.txt"
  exit $rc
fi
