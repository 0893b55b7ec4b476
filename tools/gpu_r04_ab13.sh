#!/bin/bash
# Round-4 A/B set 13: the whole GPU suite after the fused dW_hh + bias reduction launch and the deferred layer-0
# W16 rounding, then cfg2 bf16 / cfg5 fp16 steps (compare with r04ab12's *_c1 records).
set -o pipefail
OUT=gpurun_out/${1:-r04ab13}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { rc=$?; tail -40 "$OUT/pytest_gpu.log"; exit $rc; }
tail -1 "$OUT/pytest_gpu.log"
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline --no-h2d "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
run cfg2_bf16_a --no-configs --precision bf16 --steps 20
run cfg2_bf16_b --no-configs --precision bf16 --steps 20
run cfg5_fp16 --model spec_bgru --precision fp16 --steps 20
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"])
PY
