#!/bin/bash
# Round-4 A/B set 11: non-temporal C stores in the ping-pong GEMM epilogue (gemm_nt_store), cfg2 bf16 / fp32
# and cfg4 bf16; then the per-step kernel census (tools/gpu_r04_plumb.sh).
set -o pipefail
OUT=gpurun_out/${1:-r04ab11}
mkdir -p "$OUT"
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline --no-h2d "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
for m in 0 1 0 1; do
  run cfg2_bf16_nt${m}_$RANDOM "gemm_nt_store=$m" --no-configs --precision bf16 --steps 20
done
run cfg2_fp32_nt0 "gemm_nt_store=0" --no-configs --steps 20
run cfg2_fp32_nt1 "gemm_nt_store=1" --no-configs --steps 20
run cfg4_bf16_nt0 "gemm_nt_store=0" --model resnet_bgru --precision bf16 --steps 4
run cfg4_bf16_nt1 "gemm_nt_store=1" --model resnet_bgru --precision bf16 --steps 4
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items() if "gemm" in k})
PY
bash tools/gpu_r04_plumb.sh "$(basename "$OUT")_plumb"
