#!/bin/bash
# Round-4 A/B set 6: fp32 ring forward (conv_ring bit 0) on cfg3 / cfg4 fp32; g16 static priority
# (gemm16_prio) on the cfg2 GEMM shapes and the cfg2 bf16 / cfg5 fp16 steps.
set -o pipefail
OUT=gpurun_out/${1:-r04ab6}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_lowprec_gpu.py::test_gemm16_qs" \
  "tests/test_conv_gpu.py::test_conv_pool_fused_equals_separate" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for p in 0 1 0 1; do
  SRK_OPTIONS=gemm16_prio=$p timeout -k 10 120 python tools/gemm_bench.py --precision bf16 --h16 >> "$OUT/gemm_bf16_prio$p.txt" 2>&1 || exit 1
done
grep -h "^gi_l1\|^dx_l1\|^dWih_l1" "$OUT"/gemm_bf16_prio*.txt
run() {  # run TAG OPTIONS ARGS...
  local tag=$1 opt=$2; shift 2
  SRK_OPTIONS=$opt timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
}
run cfg2_bf16_p0 "gemm16_prio=0" --model mfcc_bgru --precision bf16 --steps 20
run cfg2_bf16_p1 "gemm16_prio=1" --model mfcc_bgru --precision bf16 --steps 20
run cfg5_p0 "gemm16_prio=0" --model spec_bgru --precision fp16 --steps 20
run cfg5_p1 "gemm16_prio=1" --model spec_bgru --precision fp16 --steps 20
run cfg4_r76 "conv_ring=118" --model resnet_bgru --steps 4
run cfg4_r77 "conv_ring=119" --model resnet_bgru --steps 4
run cfg3_r76 "conv_ring=118" --model fbanks_cnn --steps 10
run cfg3_r77 "conv_ring=119" --model fbanks_cnn --steps 10
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/cfg*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], r["roofline"]["kernel"], r["roofline"]["frac"])
    for k in r["roofline"]["top_kernels"][:5]:
        print("    ", k)
PY
timeout -k 10 300 python tools/gru_ab.py --variants default,prio_c0,prio_c1,prio_c0_off0,prio_c1_off0 > "$OUT/gru_ab.txt" 2>&1 || exit 1
cat "$OUT/gru_ab.txt"
