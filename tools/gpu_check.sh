#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench line, rocprofv3 kernel stats + HBM PMC passes.
#   gpurun --timeout 1100 -- bash tools/gpu_check.sh [tag]
# Every GPU step has its own time limit and the steps are chained with && (a fault ends the call).
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)"

timeout -k 10 420 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 \
  && echo "pytest gpu ok: $(tail -1 $OUT/pytest_gpu.log)" \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 240 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  && echo "bench: $(cat $OUT/bench.json)" \
  && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_stats" -o run -- \
       python3 bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
  && echo "rocprof stats ok" \
  && timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$ROOT/$OUT/prof_fetch" -o run -- \
       python3 bench.py --no-cpu-baseline --no-prof > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err" \
  && echo "pmc fetch ok" \
  && timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$ROOT/$OUT/prof_write" -o run -- \
       python3 bench.py --no-cpu-baseline --no-prof > "$OUT/bench_write.json" 2> "$OUT/bench_write.err" \
  && echo "pmc write ok"
rc=$?
echo "exit $rc"
tail -3 "$OUT/pytest_gpu.log" 2>/dev/null
exit $rc
