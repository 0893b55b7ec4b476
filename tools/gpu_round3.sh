#!/bin/bash
# Round-3 GPU evidence in one gpurun call:
#   gpurun --timeout 1150 -- bash tools/gpu_round3.sh TAG
# pytest -m gpu, smoke, the default bench line (cfg2 headline + cfg3/4/5 records + CPU baseline),
# rocprofv3 --kernel-trace --stats of the default bench command, and separate FETCH_SIZE / WRITE_SIZE
# PMC passes per config command (eager steps: the same kernels as the graph replays).  Every GPU step
# has its own time limit; steps are chained with && (a failure ends the call).
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "host: $(grep -m1 'model name' /proc/cpuinfo)"
stats() {   # stats NAME ARGS...: kernel-trace stats of one config's bench command (graph replays)
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/stats_${name}" -o run -- \
    python3 bench.py --no-cpu-baseline --no-configs --no-feature-roofline "$@" \
    > "$OUT/stats_${name}.json" 2> "$OUT/stats_${name}.err" \
  && python3 tools/rocpd_summary.py "$OUT/stats_${name}" > "$OUT/summary_${name}_stats.txt" && rm -rf "$OUT/stats_${name}"
}
pmc() {   # pmc NAME COUNTER ARGS...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d "$ROOT/$OUT/pmc_${name}_${ctr}" -o run -- \
    python3 bench.py --no-cpu-baseline --no-prof --no-configs --no-feature-roofline --no-graph "$@" \
    > "$OUT/pmc_${name}_${ctr}.json" 2> "$OUT/pmc_${name}_${ctr}.err"
}
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; } \
  && echo "pytest gpu: $(tail -1 $OUT/pytest_gpu.log 2>/dev/null)" \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && echo "smoke: $(tail -1 $OUT/smoke.log)" \
  && timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  && echo "bench ok" \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_stats" -o run -- \
       python3 bench.py --no-cpu-baseline --no-feature-roofline --no-configs > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
  && stats cfg3 --model fbanks_cnn --no-lowprec --steps 10 && stats cfg4 --model resnet_bgru --no-lowprec --steps 4 \
  && stats cfg5 --model spec_bgru --precision fp16 --steps 20 \
  && echo "stats ok" \
  && pmc cfg2 FETCH_SIZE && pmc cfg2 WRITE_SIZE \
  && pmc cfg3 FETCH_SIZE --model fbanks_cnn --no-lowprec --steps 10 && pmc cfg3 WRITE_SIZE --model fbanks_cnn --no-lowprec --steps 10 \
  && pmc cfg4 FETCH_SIZE --model resnet_bgru --no-lowprec --steps 4 && pmc cfg4 WRITE_SIZE --model resnet_bgru --no-lowprec --steps 4 \
  && pmc cfg5 FETCH_SIZE --model spec_bgru --precision fp16 --steps 20 && pmc cfg5 WRITE_SIZE --model spec_bgru --precision fp16 --steps 20 \
  && echo "pmc ok" \
  && python3 tools/rocpd_summary.py "$OUT/prof_stats" --fetch "$OUT/pmc_cfg2_FETCH_SIZE" --write "$OUT/pmc_cfg2_WRITE_SIZE" \
       > "$OUT/summary_cfg2.txt" \
  && python3 tools/pmc_traffic.py "$OUT/pmc_cfg2_FETCH_SIZE" "$OUT/pmc_cfg2_WRITE_SIZE" --model mfcc_bgru --batch 256 \
       --precisions fp32,bf16 --source "$TAG cfg2" -o "$OUT/pmc_traffic_mfcc_bgru.json" > /dev/null \
  && python3 tools/pmc_traffic.py "$OUT/pmc_cfg3_FETCH_SIZE" "$OUT/pmc_cfg3_WRITE_SIZE" --model fbanks_cnn --batch 512 \
       --precisions fp32 --source "$TAG cfg3" -o "$OUT/pmc_traffic_fbanks_cnn.json" > /dev/null \
  && python3 tools/pmc_traffic.py "$OUT/pmc_cfg4_FETCH_SIZE" "$OUT/pmc_cfg4_WRITE_SIZE" --model resnet_bgru --batch 512 \
       --precisions fp32 --source "$TAG cfg4" -o "$OUT/pmc_traffic_resnet_bgru.json" > /dev/null \
  && python3 tools/pmc_traffic.py "$OUT/pmc_cfg5_FETCH_SIZE" "$OUT/pmc_cfg5_WRITE_SIZE" --model spec_bgru --batch 512 \
       --precisions fp16 --source "$TAG cfg5" -o "$OUT/pmc_traffic_spec_bgru.json" > /dev/null \
  && for c in cfg3 cfg4 cfg5; do python3 tools/rocpd_summary.py "$OUT/pmc_${c}_FETCH_SIZE" --fetch "$OUT/pmc_${c}_FETCH_SIZE" \
       --write "$OUT/pmc_${c}_WRITE_SIZE" > "$OUT/summary_${c}_pmc.txt" || exit 1; done \
  && echo "summaries ok"
rc=$?
# the rocpd databases exceed what gpurun copies back: keep the summaries only
rm -rf "$OUT"/prof_stats "$OUT"/pmc_cfg*_FETCH_SIZE "$OUT"/pmc_cfg*_WRITE_SIZE
echo "exit $rc"
exit $rc
