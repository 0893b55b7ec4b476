#!/bin/bash
# Round-4 A/B set 14: GEMM swizzle group height (SRK_GROUP_M: tile rows per L2 group; default = sqrt(32 per_cu
# BN / BM) = 4 for the 256 x 128 fp32 tiles) on the cfg2 fp32 step: whole-step time, and FETCH_SIZE per GEMM
# kernel (the x W^T projection moves 2.4x its algorithmic bytes).
set -o pipefail
OUT=gpurun_out/${1:-r04ab14}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for g in 4 8 16 2; do
  SRK_GROUP_M=$g timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline --no-h2d \
    --no-configs --steps 20 > "$OUT/cfg2_fp32_g$g.json" 2> "$OUT/cfg2_fp32_g$g.err" || exit $?
  SRK_GROUP_M=$g timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$ROOT/$OUT/pmc_g$g" -o run -- \
    python3 bench.py --no-cpu-baseline --no-prof --no-configs --no-feature-roofline --no-h2d --no-graph --no-lowprec \
    --steps 3 > "$OUT/pmc_g$g.json" 2> "$OUT/pmc_g$g.err" || exit $?
  python3 tools/rocpd_summary.py "$OUT/pmc_g$g" --fetch "$OUT/pmc_g$g" > "$OUT/summary_g$g.txt" && rm -rf "$OUT/pmc_g$g" || exit $?
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/cfg2_*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items() if "gemm" in k})
PY
