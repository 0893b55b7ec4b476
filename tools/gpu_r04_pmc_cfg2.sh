#!/bin/bash
# cfg2 FETCH_SIZE / WRITE_SIZE passes only (the fp32 x W^T GEMM traffic check):
#   gpurun -- bash tools/gpu_r04_pmc_cfg2.sh TAG
set -o pipefail
TAG=${1:-r04p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
pmc() {   # pmc NAME COUNTER ARGS...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d "$ROOT/$OUT/pmc_${name}_${ctr}" -o run -- \
    python3 bench.py --no-cpu-baseline --no-prof --no-configs --no-feature-roofline --no-h2d --no-graph "$@" \
    > "$OUT/pmc_${name}_${ctr}.json" 2> "$OUT/pmc_${name}_${ctr}.err"
}
pmc cfg2 FETCH_SIZE && pmc cfg2 WRITE_SIZE \
  && python3 tools/pmc_traffic.py "$OUT/pmc_cfg2_FETCH_SIZE" "$OUT/pmc_cfg2_WRITE_SIZE" --model mfcc_bgru --batch 256 \
       --precisions fp32,bf16 --source "$TAG cfg2" -o "$OUT/pmc_traffic_mfcc_bgru.json" > /dev/null \
  && python3 tools/rocpd_summary.py "$OUT/pmc_cfg2_FETCH_SIZE" --fetch "$OUT/pmc_cfg2_FETCH_SIZE" \
       --write "$OUT/pmc_cfg2_WRITE_SIZE" > "$OUT/summary_cfg2_pmc.txt"
rc=$?
rm -rf "$OUT"/pmc_cfg2_FETCH_SIZE "$OUT"/pmc_cfg2_WRITE_SIZE
exit $rc
