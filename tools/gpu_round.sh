#!/bin/bash
# Full round-end GPU evidence in one gpurun call:
#   gpurun --timeout 1150 -- bash tools/gpu_round.sh TAG
# pytest -m gpu, smoke, the default bench line (with CPU baseline), the other configs' bench lines,
# rocprofv3 --kernel-trace --stats of the default bench, and separate FETCH_SIZE / WRITE_SIZE PMC
# passes.  Every GPU step has its own time limit; steps are chained with && (a failure ends it).
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "host: $(grep -m1 'model name' /proc/cpuinfo)"
timeout -k 10 420 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 \
  && echo "pytest gpu: $(tail -1 $OUT/pytest_gpu.log)" \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && echo "smoke: $(tail -1 $OUT/smoke.log)" \
  && timeout -k 10 240 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  && echo "bench: $(cat $OUT/bench.json)" \
  && for m in fbanks_cnn resnet_bgru spec_bgru mfrn_bgru; do
       timeout -k 10 300 python bench.py --model $m --steps 10 > "$OUT/bench_$m.json" 2> "$OUT/bench_$m.err" || exit 1
     done \
  && timeout -k 10 300 python bench.py --model spec_bgru --precision fp16 --steps 10 --no-cpu-baseline \
       > "$OUT/bench_spec_bgru_fp16.json" 2> "$OUT/bench_spec_bgru_fp16.err" \
  && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_stats" -o run -- \
       python3 bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
  && timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$ROOT/$OUT/prof_fetch" -o run -- \
       python3 bench.py --no-cpu-baseline --no-prof > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err" \
  && timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$ROOT/$OUT/prof_write" -o run -- \
       python3 bench.py --no-cpu-baseline --no-prof > "$OUT/bench_write.json" 2> "$OUT/bench_write.err" \
  && echo "profiles ok"
rc=$?
echo "exit $rc"
exit $rc
