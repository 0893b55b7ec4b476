#!/bin/bash
# Round-4 A/B set 3: the 16-bit ring convolutions (conv_ring bits 4-6) on cfg3 / cfg4 in bf16.
set -o pipefail
OUT=gpurun_out/${1:-r04ab3}
mkdir -p "$OUT"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
}
run cfg3_bf16_noring "" --model fbanks_cnn --precision bf16 --steps 10
run cfg3_bf16_ring "conv_ring=118" --model fbanks_cnn --precision bf16 --steps 10
run cfg4_bf16_noring "" --model resnet_bgru --precision bf16 --steps 4
run cfg4_bf16_ring "conv_ring=118" --model resnet_bgru --precision bf16 --steps 4
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 2) for k, v in r["kernels"].items() if k.startswith("conv")})
    for k in r["roofline"]["top_kernels"][:4]:
        print("    ", k)
PY
