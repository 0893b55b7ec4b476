#!/bin/bash
# Round-4 A/B set 8: the fused dW_hh parity (A/B 7's test) and the forward worker waves (gru_fwd_worker):
# bitwise test, then cfg2 bf16 / mfrn bf16 steps with the new options on and off.
set -o pipefail
OUT=gpurun_out/${1:-r04ab8}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_lowprec_gpu.py::test_bigru_dwhh_fused_matches_gemm" "tests/test_lowprec_gpu.py::test_bigru_fwd_worker" \
  > "$OUT/pytest_new.log" 2>&1 || { rc=$?; tail -40 "$OUT/pytest_new.log"; exit $rc; }
tail -3 "$OUT/pytest_new.log"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
run cfg2_bf16_dw0_ow0 "gru_dwhh_fused=0,gru_fwd_worker=0" --model mfcc_bgru --precision bf16 --steps 20
run cfg2_bf16_dw1_ow0 "gru_dwhh_fused=1,gru_fwd_worker=0" --model mfcc_bgru --precision bf16 --steps 20
run cfg2_bf16_dw1_ow1 "gru_dwhh_fused=1,gru_fwd_worker=1" --model mfcc_bgru --precision bf16 --steps 20
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items()})
    for k in r["roofline"]["top_kernels"][:4]:
        print("    ", k)
PY
