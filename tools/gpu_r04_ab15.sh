#!/bin/bash
# Round-4 A/B set 15: GEMM kernel choice re-measured at the final code — fp32: register-staged 256 x 128
# (default for x W^T) vs the ping-pong kernel everywhere (gemm32_kernel=2); 16-bit: the ping-pong g16
# (default) vs the register-staged h16 everywhere (gemm16_kernel=1).
set -o pipefail
OUT=gpurun_out/${1:-r04ab15}
mkdir -p "$OUT"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline --no-h2d \
    --no-configs "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
for i in 1 2; do
  run fp32_k0_$i "gemm32_kernel=0" --steps 20
  run fp32_k2_$i "gemm32_kernel=2" --steps 20
  run bf16_k0_$i "gemm16_kernel=0" --precision bf16 --steps 20
  run bf16_k1_$i "gemm16_kernel=1" --precision bf16 --steps 20
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    top = [(k["kernel"][:60], round(k["ms_total"], 3)) for k in r["roofline"]["top_kernels"] if "gemm" in k["kernel"]]
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items() if "gemm" in k}, top)
PY
