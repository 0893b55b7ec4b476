#!/bin/bash
# Round-6 GPU evidence:  gpurun --timeout 1150 -- bash tools/gpu_round6.sh TAG
# pytest -m gpu, smoke, the default bench line, rocprofv3 --kernel-trace --stats of the cfg2 bench
# command and of each config command (graph replays), summarised on the box.  Every GPU step has its
# own time limit; steps are chained with && (a failure ends the call).
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "host: $(grep -m1 'model name' /proc/cpuinfo)"
stats() {   # stats NAME ARGS...: kernel-trace stats of one config's bench command (graph replays)
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/stats_${name}" -o run -- \
    python3 bench.py --no-cpu-baseline --no-configs --no-feature-roofline --no-h2d "$@" \
    > "$OUT/stats_${name}.json" 2> "$OUT/stats_${name}.err" \
  && python3 tools/rocpd_summary.py "$OUT/stats_${name}" > "$OUT/summary_${name}_stats.txt" && rm -rf "$OUT/stats_${name}"
}
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; } \
  && echo "pytest gpu: $(tail -1 $OUT/pytest_gpu.log 2>/dev/null)" \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && echo "smoke: $(tail -1 $OUT/smoke.log)" \
  && timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  && echo "bench ok" \
  && stats cfg2 && stats cfg3 --model fbanks_cnn --no-lowprec --steps 10 \
  && stats cfg4 --model resnet_bgru --no-lowprec --steps 4 && stats cfg5 --model spec_bgru --precision fp16 --steps 20 \
  && stats mfrn --model mfrn_bgru --no-lowprec --steps 10 \
  && stats cfg3b --model fbanks_cnn --precision bf16 --no-lowprec --steps 10 \
  && stats cfg4b --model resnet_bgru --precision bf16 --no-lowprec --steps 4 \
  && echo "stats ok"
rc=$?
rm -rf "$OUT"/stats_cfg2 "$OUT"/stats_cfg3 "$OUT"/stats_cfg4 "$OUT"/stats_cfg5 "$OUT"/stats_cfg3b "$OUT"/stats_cfg4b "$OUT"/stats_mfrn
echo "exit $rc"
exit $rc
