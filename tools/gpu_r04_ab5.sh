#!/bin/bash
# Round-4 A/B set 5: conv tests after the 16-bit ring default (0x76) and the direct 16-bit unpool
# (conv_unpool16), then cfg3 / cfg4 bf16 steps with conv_unpool16 1 vs 0.
set -o pipefail
OUT=gpurun_out/${1:-r04ab5}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests \
  > "$OUT/pytest_conv.log" 2>&1 || { tail -40 "$OUT/pytest_conv.log"; exit 1; }
tail -2 "$OUT/pytest_conv.log"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
}
run cfg3_bf16_u1 "conv_unpool16=1" --model fbanks_cnn --precision bf16 --steps 10
run cfg3_bf16_u0 "conv_unpool16=0" --model fbanks_cnn --precision bf16 --steps 10
run cfg4_bf16 "" --model resnet_bgru --precision bf16 --steps 4
run cfg3_fp32 "" --model fbanks_cnn --steps 10
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/cfg*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 2) for k, v in r["kernels"].items()})
    for k in r["roofline"]["top_kernels"][:5]:
        print("    ", k)
PY
