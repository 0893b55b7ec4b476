#!/bin/bash
# Per-step kernel census of the cfg2 bf16 / fp32 graph-replayed steps (200 replays dominate the counts):
# which non-GEMM / non-recurrence launches (memsets, torch fills / copies, reductions) remain per step.
set -o pipefail
OUT=gpurun_out/${1:-r04plumb}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for p in bf16 fp32; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/st_$p" -o run -- \
    python3 bench.py --no-cpu-baseline --no-configs --no-feature-roofline --no-h2d --no-lowprec --no-prof \
    --precision $p --steps 200 > "$OUT/b_$p.json" 2> "$OUT/b_$p.err" \
  && python3 tools/rocpd_summary.py "$OUT/st_$p" > "$OUT/summary_$p.txt" && rm -rf "$OUT/st_$p" || exit $?
done
