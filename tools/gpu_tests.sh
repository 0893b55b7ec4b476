#!/bin/bash
# One gpurun call: the GPU test suite (or a subset) with per-test timeouts, then one bench line.
#   gpurun --timeout 900 -- bash tools/gpu_tests.sh TAG [pytest selection args...]
set -o pipefail
TAG=${1:-t}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${@:-tests}" > "$OUT/pytest.log" 2>&1
rc=$?
tail -1 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|^E " "$OUT/pytest.log" | head -40; exit $rc; fi
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json"
