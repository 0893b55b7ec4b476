#!/bin/bash
# SQ / GRBM counters of the 16-bit GEMM kernels on the cfg2 layer-1 shapes (tools/gemm_bench.py), one
# rocprofv3 pass per counter group (<= 8 SQ counters each), then the per-kernel summary table.
#   gpurun --timeout 600 -- bash tools/gemm_pmc.sh TAG [KERNEL16]
set -o pipefail
TAG=${1:-gemm_pmc}
K16=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc -d "$ROOT/$OUT/p${i}_gemm" -o run -- \
    python3 tools/gemm_bench.py --precision ${PREC:-bf16} $([ "${PREC:-bf16}" = fp32 ] || echo --h16) --kernel16 $K16 --reps 3 > "$OUT/p${i}.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p${i}.log"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && rm -rf "$OUT"/p[0-9]*_gemm && cat "$OUT/summary.txt"
