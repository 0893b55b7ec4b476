#!/bin/bash
# Round-4 A/B set 16: conv weights re-laid-out straight into their 16-bit copies (weight_layout16_kernel):
# the conv / 16-bit / config-batch parity tests, then cfg3 / cfg4 bf16 steps (compare r04h_bench.json).
set -o pipefail
OUT=gpurun_out/${1:-r04ab16}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_lowprec_gpu.py tests/test_bn_copy16_gpu.py tests/test_config_batch_gpu.py tests/test_models_gpu.py \
  > "$OUT/pytest.log" 2>&1 || { rc=$?; tail -40 "$OUT/pytest.log"; exit $rc; }
tail -1 "$OUT/pytest.log"
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline --no-h2d "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
run cfg3_bf16 --model fbanks_cnn --precision bf16 --steps 10
run cfg4_bf16 --model resnet_bgru --precision bf16 --steps 4
run mfrn_bf16 --model mfrn_bgru --precision bf16 --steps 10
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items() if "conv" in k})
PY
