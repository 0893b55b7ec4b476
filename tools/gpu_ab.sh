#!/bin/bash
# A/B of srk options on one bench command:  gpurun -- bash tools/gpu_ab.sh TAG "BENCH ARGS" "opt=a,opt2=b" "opt=c" ...
# An empty option string is the default build.  Prints value / ms per step for each, twice (ABAB order).
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for opts in "$@"; do
    i=$((i + 1))
    SRK_OPTIONS="$opts" timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs --no-feature-roofline --no-h2d $ARGS \
      > "$OUT/ab_${i}_$rep.json" 2> "$OUT/ab_${i}_$rep.err" || { echo "run failed: [$opts]"; tail -5 "$OUT/ab_${i}_$rep.err"; exit 1; }
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('[%s] rep %s: %s %s  %s ms' % (sys.argv[2], sys.argv[3], r['value'], r['unit'], r['ms_per_step']))" "$OUT/ab_${i}_$rep.json" "$opts" "$rep"
  done
done
