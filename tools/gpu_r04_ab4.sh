#!/bin/bash
# Round-4 A/B set 4 (one gpurun call): new GPU tests (DP step graph with captured all-reduces, g16
# 32-deep sections), the 16-bit GEMM sections (gemm16_qs 1 vs 2) on the cfg2 shapes and the cfg2 /
# cfg5 steps, then A/B set 3 (16-bit ring convs) and the cfg2 PMC traffic passes.
set -o pipefail
OUT=gpurun_out/${1:-r04ab4}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dp_graph_gpu.py \
  "tests/test_lowprec_gpu.py::test_gemm16_qs" > "$OUT/pytest_new.log" 2>&1 || { tail -30 "$OUT/pytest_new.log"; exit 1; }
tail -2 "$OUT/pytest_new.log"
for qs in 1 2 1 2; do
  SRK_OPTIONS=gemm16_qs=$qs timeout -k 10 120 python tools/gemm_bench.py --precision bf16 --h16 >> "$OUT/gemm_bf16_qs$qs.txt" 2>&1 || exit 1
done
grep -h "^gi_l1\|^dx_l1\|^dWih_l1" "$OUT"/gemm_bf16_qs*.txt
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
}
run cfg2_bf16_qs1 "gemm16_qs=1" --model mfcc_bgru --precision bf16 --steps 20
run cfg2_bf16_qs2 "gemm16_qs=2" --model mfcc_bgru --precision bf16 --steps 20
run cfg5_qs1 "gemm16_qs=1" --model spec_bgru --precision fp16 --steps 20
run cfg5_qs2 "gemm16_qs=2" --model spec_bgru --precision fp16 --steps 20
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/cfg*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], r["roofline"]["kernel"], r["roofline"]["frac"])
PY
bash tools/gpu_r04_ab3.sh r04ab3 > "$OUT/ab3.txt" 2>&1 || { echo "ab3 failed"; exit 1; }
cat "$OUT/ab3.txt"
bash tools/gpu_r04_pmc_cfg2.sh r04p && echo "pmc ok"
