#!/bin/bash
# SQ / GRBM / TCC counters of the conv kernels on the bench shapes (tools/conv_bench.py), one rocprofv3 pass per
# counter group (<= 8 SQ counters each), then the per-kernel summary table (tools/pmc_table.py).
#   gpurun --timeout 600 -- bash tools/conv_pmc.sh TAG "fb_conv2,rn_l4" [bf16]
set -o pipefail
TAG=${1:-conv_pmc}
ONLY=${2:-fb_conv2}
PREC=${3:-bf16}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc -d "$ROOT/$OUT/p${i}_conv" -o run -- \
    python3 tools/conv_bench.py --prec $PREC --only $ONLY > "$OUT/p${i}.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p${i}.log"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && rm -rf "$OUT"/p[0-9]*_conv && cat "$OUT/summary.txt"
