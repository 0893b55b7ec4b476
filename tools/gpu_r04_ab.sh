#!/bin/bash
# Round-4 A/B measurements (one gpurun call):
#   GEMM swizzle group size on the cfg2 GEMM shapes (SRK_GROUP_M=8: round 3's value, 0: balanced),
#   conv tile shape on the cfg3 step (SRK_OPTIONS conv_tile=128 / 256).
set -o pipefail
OUT=gpurun_out/${1:-r04ab}
mkdir -p "$OUT"
for g in 8 0; do
  for prec in fp32 bf16; do
    extra=""; [ $prec = bf16 ] && extra="--h16"
    SRK_GROUP_M=$g timeout -k 10 120 python tools/gemm_bench.py --precision $prec $extra > "$OUT/gemm_${prec}_g$g.txt" 2>&1 || exit 1
  done
done
SRK_GROUP_M=0 timeout -k 10 120 python tools/gemm_bench.py --precision fp32 --kernel32 2 > "$OUT/gemm_fp32_k2.txt" 2>&1 || exit 1
for sk in 0 1; do
  SRK_OPTIONS=gemm_streamk=$sk timeout -k 10 120 python tools/gemm_bench.py --precision fp32 > "$OUT/gemm_fp32_sk$sk.txt" 2>&1 || exit 1
done
for pers in 0 1; do
  SRK_OPTIONS=gemm16_persistent=$pers timeout -k 10 120 python tools/gemm_bench.py --precision bf16 --h16 > "$OUT/gemm_bf16_pers$pers.txt" 2>&1 || exit 1
done
for t in 128 256 ring; do
  opt="conv_tile=$t"; [ $t = ring ] && opt="conv_ring=1"
  SRK_OPTIONS=$opt timeout -k 10 200 python bench.py --model fbanks_cnn --no-lowprec --no-cpu-baseline \
    --no-feature-roofline --steps 10 > "$OUT/cfg3_tile$t.json" 2> "$OUT/cfg3_tile$t.err" || exit 1
done
for v in 0 1 2 3 0 1 2 3; do
  SRK_OPTIONS=mfcc_variant=$v FEAT_ONLY=mfcc timeout -k 10 120 python tools/feat_bench.py >> "$OUT/mfcc_var$v.txt" 2>&1 || exit 1
done
tail -n 12 "$OUT"/gemm_*.txt
tail -n 2 "$OUT"/mfcc_var*.txt
python - "$OUT" <<'PY'
import json, sys
for t in (128, 256, "ring"):
    r = json.loads(open("%s/cfg3_tile%s.json" % (sys.argv[1], t)).read().strip().splitlines()[-1])
    print("cfg3 conv %s: %.1f utt/s, %.3f ms/step" % (t, r["value"], r["ms_per_step"]))
    for k in r["roofline"]["top_kernels"]:
        print("   ", k)
PY
