#!/bin/bash
# K1 per-phase instruction budget (VERDICT r04 "next" #3): SQ_INSTS_* per clip of the product mfcc3_kernel
# and of the SRK_MFCC_STOP=0..3 diagnostic builds (tools/build_variant.sh stopN -DSRK_MFCC_STOP=N, SRCS=features),
# on 65,536 clips; the phase counts are the differences (tools/feat_budget.py).
#   gpurun --timeout 600 -- bash tools/feat_budget.sh TAG
set -o pipefail
TAG=${1:-budget}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in stop0 stop1 stop2 stop3 full; do
  lib=""
  [ "$v" != full ] && lib="$ROOT/tools/_exp/libsrk_$v.so"
  SRK_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $PMC -d "$ROOT/$OUT/$v" -o run -- \
    python3 tools/mfcc_only.py mfcc 65536 > "$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
done
python3 tools/feat_budget.py "$OUT" | tee "$OUT/budget.txt" && rm -rf "$OUT"/stop* "$OUT"/full
