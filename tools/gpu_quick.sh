#!/bin/bash
# Quick GPU check of a change set:  gpurun --timeout 900 -- bash tools/gpu_quick.sh TAG "pytest selection..." [bench args]
# pytest on the given selection, then (if BENCH is set) a bench line with those args.
set -o pipefail
TAG=${1:-quick}
SEL=${2:-tests -m gpu}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $SEL -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?
  echo "bench rc=$rc"; tail -c 600 "$OUT/bench.json"
  exit $rc
fi
