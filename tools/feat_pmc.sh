#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each) and VALU / LDS / wait counters (two SQ groups)
# of the feature kernels (K1-K3) on 65,536 clips, one rocprofv3 pass per group, then the summaries:
# DIR/summary.txt (every counter per dispatch) and DIR/pmc_feature.json (bench.py feature_roofline).
#   gpurun --timeout 600 -- bash tools/feat_pmc.sh TAG
set -o pipefail
TAG=${1:-feat}
OUT=gpurun_out/$TAG
CLIPS=${CLIPS:-65536}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES"; do
  i=$((i+1))
  for k in ${KERNELS:-mfcc fbank spec}; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc -d "$ROOT/$OUT/p${i}_$k" -o run -- \
      python3 tools/mfcc_only.py $k $CLIPS > "$OUT/p${i}_$k.log" 2>&1 || { echo "pass $i $k failed"; tail -5 "$OUT/p${i}_$k.log"; exit 1; }
    echo "pass $i $k ok"
  done
done
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && \
python3 tools/feat_pmc.py "$OUT" --clips $CLIPS --source "tools/feat_pmc.sh $TAG" -o "$OUT/pmc_feature.json" && \
rm -rf "$OUT"/p[0-9]* && cat "$OUT/summary.txt"
