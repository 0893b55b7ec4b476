#!/bin/bash
# Round-4 A/B, second set: cfg3 / cfg4 with the ring conv defaults, the pooled conv's backward through
# the unpooling gathers (default) vs the dense scratch gradient on the ring kernels.
set -o pipefail
OUT=gpurun_out/${1:-r04ab2}
mkdir -p "$OUT"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
}
run cfg3_default "" --model fbanks_cnn --steps 10
run cfg3_dense "conv_unpool_gather=0" --model fbanks_cnn --steps 10
run cfg3_noring "conv_ring=0" --model fbanks_cnn --steps 10
run cfg4_default "" --model resnet_bgru --steps 4
run cfg4_noring "conv_ring=0" --model resnet_bgru --steps 4
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 2) for k, v in r["kernels"].items() if k.startswith("conv")})
PY
