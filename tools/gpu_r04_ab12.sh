#!/bin/bash
# Round-4 A/B set 12: BiGRU layer hand-over of the 16-bit h copy (srk_gru_layer_fwd_x16; SRK_BN_COPY16 switches
# every producer copy): parity tests, then cfg2 bf16 / cfg5 fp16 steps with and without.
set -o pipefail
OUT=gpurun_out/${1:-r04ab12}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_copy16_gpu.py \
  tests/test_lowprec_gpu.py tests/test_models_gpu.py > "$OUT/pytest.log" 2>&1 || { rc=$?; tail -40 "$OUT/pytest.log"; exit $rc; }
tail -3 "$OUT/pytest.log"
run() {  # run TAG BN_COPY16 ARGS...
  local tag=$1 on=$2; shift 2
  SRK_BN_COPY16=$on timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline --no-h2d "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
for on in 0 1 0 1; do
  run cfg2_bf16_c${on}_$RANDOM $on --no-configs --precision bf16 --steps 20
done
run cfg5_fp16_c0 0 --model spec_bgru --precision fp16 --steps 20
run cfg5_fp16_c1 1 --model spec_bgru --precision fp16 --steps 20
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"])
PY
