#!/bin/bash
# PMC counter evidence at the current build:  gpurun --timeout 1150 -- bash tools/gpu_pmc.sh TAG [traffic|feature|all]
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs, --kernel-trace only beside --pmc; eager steps:
# the same kernels as the graph replays) of every config command the default bench line carries, summarised
# on the box by tools/pmc_traffic.py into pmc_traffic_<model>.json — each stamped with the loaded library's
# srk_source_stamp(), which bench.py requires to match before it attaches a traffic figure.  "feature" runs
# the K1-K3 counter passes instead (tools/feat_pmc.sh), "all" both.  Copy the JSON files into profiles/.
set -o pipefail
TAG=${1:-pmc}
WHAT=${2:-traffic}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
pmc() {   # pmc NAME COUNTER ARGS...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d "$ROOT/$OUT/pmc_${name}_${ctr}" -o run -- \
    python3 bench.py --no-cpu-baseline --no-prof --no-configs --no-feature-roofline --no-h2d --no-graph "$@" \
    > "$OUT/pmc_${name}_${ctr}.json" 2> "$OUT/pmc_${name}_${ctr}.err" && echo "pmc $name $ctr ok"
}
traffic() {   # traffic NAME MODEL BATCH PRECISIONS [--merge]
  python3 tools/pmc_traffic.py "$OUT/pmc_$1_FETCH_SIZE" "$OUT/pmc_$1_WRITE_SIZE" --model $2 --batch $3 \
    --precisions $4 --source "$TAG $1" -o "$OUT/pmc_traffic_$2.json" $5 > /dev/null \
  && python3 tools/rocpd_summary.py "$OUT/pmc_$1_FETCH_SIZE" --fetch "$OUT/pmc_$1_FETCH_SIZE" \
       --write "$OUT/pmc_$1_WRITE_SIZE" > "$OUT/summary_$1_pmc.txt" \
  && rm -rf "$OUT/pmc_$1_FETCH_SIZE" "$OUT/pmc_$1_WRITE_SIZE"
}
both() {   # both NAME ARGS...
  local name=$1; shift
  pmc $name FETCH_SIZE "$@" && pmc $name WRITE_SIZE "$@"
}
rc=0
if [ "$WHAT" != "feature" ]; then
  both cfg2 --steps 10 && traffic cfg2 mfcc_bgru 256 fp32,bf16 \
    && both cfg3 --model fbanks_cnn --no-lowprec --steps 6 && traffic cfg3 fbanks_cnn 512 fp32 \
    && both cfg3b --model fbanks_cnn --precision bf16 --no-lowprec --steps 6 \
    && traffic cfg3b fbanks_cnn 512 bf16 --merge \
    && both cfg4 --model resnet_bgru --no-lowprec --steps 3 && traffic cfg4 resnet_bgru 512 fp32 \
    && both cfg4b --model resnet_bgru --precision bf16 --no-lowprec --steps 3 \
    && traffic cfg4b resnet_bgru 512 bf16 --merge \
    && both cfg5 --model spec_bgru --precision fp16 --steps 10 && traffic cfg5 spec_bgru 512 fp16 \
    && both mfrn --model mfrn_bgru --no-lowprec --steps 6 && traffic mfrn mfrn_bgru 256 fp32 \
    && echo "traffic ok"
  rc=$?
fi
if [ $rc -eq 0 ] && { [ "$WHAT" = "feature" ] || [ "$WHAT" = "all" ]; }; then
  bash tools/feat_pmc.sh "$TAG/feat" && cp "$OUT/feat/pmc_feature.json" "$OUT/pmc_feature.json"
  rc=$?
fi
rm -rf "$OUT"/pmc_*_FETCH_SIZE "$OUT"/pmc_*_WRITE_SIZE
echo "exit $rc"
exit $rc
