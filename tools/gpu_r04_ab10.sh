#!/bin/bash
# Round-4 A/B set 10: fused dW_hh timing variants (gru_dwhh_fused bits 1 / 2) on cfg2 bf16, then A/B set 9
# (BatchNorm-emitted 16-bit conv operands).
set -o pipefail
OUT=gpurun_out/${1:-r04ab10}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_lowprec_gpu.py::test_bigru_dwhh_fused_matches_gemm" > "$OUT/pytest_dw.log" 2>&1 \
  || { rc=$?; tail -40 "$OUT/pytest_dw.log"; exit $rc; }
tail -3 "$OUT/pytest_dw.log"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
for m in 0 1 3 5 7 0 1; do
  run cfg2_bf16_dw${m}_$RANDOM "gru_dwhh_fused=$m" --model mfcc_bgru --precision bf16 --steps 20
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items()})
PY
bash tools/gpu_r04_ab9.sh "$(basename "$OUT")_bn"
