#!/bin/bash
# Round-4 GPU evidence, call 2 of 2:  gpurun --timeout 1150 -- bash tools/gpu_round4_pmc.sh TAG
# FETCH_SIZE / WRITE_SIZE passes per config command (separate rocprofv3 runs, --kernel-trace only
# beside --pmc; eager steps: the same kernels as the graph replays), summarised on the box into
# profiles/pmc_traffic_<model>.json form by tools/pmc_traffic.py.
set -o pipefail
TAG=${1:-r04}
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
traffic() {   # traffic NAME MODEL BATCH PRECISIONS [--merge]
  python3 tools/pmc_traffic.py "$OUT/pmc_$1_FETCH_SIZE" "$OUT/pmc_$1_WRITE_SIZE" --model $2 --batch $3 \
    --precisions $4 --source "$TAG $1" -o "$OUT/pmc_traffic_$2.json" $5 > /dev/null \
  && python3 tools/rocpd_summary.py "$OUT/pmc_$1_FETCH_SIZE" --fetch "$OUT/pmc_$1_FETCH_SIZE" \
       --write "$OUT/pmc_$1_WRITE_SIZE" > "$OUT/summary_$1_pmc.txt"
}
pmc cfg2 FETCH_SIZE && pmc cfg2 WRITE_SIZE && traffic cfg2 mfcc_bgru 256 fp32,bf16 \
  && pmc cfg3 FETCH_SIZE --model fbanks_cnn --no-lowprec --steps 10 && pmc cfg3 WRITE_SIZE --model fbanks_cnn --no-lowprec --steps 10 \
  && traffic cfg3 fbanks_cnn 512 fp32 \
  && pmc cfg3b FETCH_SIZE --model fbanks_cnn --precision bf16 --no-lowprec --steps 10 \
  && pmc cfg3b WRITE_SIZE --model fbanks_cnn --precision bf16 --no-lowprec --steps 10 \
  && traffic cfg3b fbanks_cnn 512 bf16 --merge \
  && pmc cfg4 FETCH_SIZE --model resnet_bgru --no-lowprec --steps 4 && pmc cfg4 WRITE_SIZE --model resnet_bgru --no-lowprec --steps 4 \
  && traffic cfg4 resnet_bgru 512 fp32 \
  && pmc cfg4b FETCH_SIZE --model resnet_bgru --precision bf16 --no-lowprec --steps 4 \
  && pmc cfg4b WRITE_SIZE --model resnet_bgru --precision bf16 --no-lowprec --steps 4 \
  && traffic cfg4b resnet_bgru 512 bf16 --merge \
  && pmc cfg5 FETCH_SIZE --model spec_bgru --precision fp16 --steps 20 && pmc cfg5 WRITE_SIZE --model spec_bgru --precision fp16 --steps 20 \
  && traffic cfg5 spec_bgru 512 fp16 \
  && pmc mfrn FETCH_SIZE --model mfrn_bgru --no-lowprec --steps 10 && pmc mfrn WRITE_SIZE --model mfrn_bgru --no-lowprec --steps 10 \
  && traffic mfrn mfrn_bgru 256 fp32 \
  && echo "pmc ok"
rc=$?
rm -rf "$OUT"/pmc_cfg*_FETCH_SIZE "$OUT"/pmc_cfg*_WRITE_SIZE "$OUT"/pmc_mfrn_*_SIZE
echo "exit $rc"
exit $rc
