#!/bin/bash
# Round-4 A/B measurements (one gpurun call): GEMM swizzle group size on the cfg2 shapes.
set -o pipefail
OUT=gpurun_out/${1:-r04ab}
mkdir -p "$OUT"
for g in 8 0; do
  for prec in fp32 bf16; do
    extra=""; [ $prec = bf16 ] && extra="--h16"
    SRK_GROUP_M=$g timeout -k 10 120 python tools/gemm_bench.py --precision $prec $extra > "$OUT/gemm_${prec}_g$g.txt" 2>&1 || exit 1
  done
done
tail -n 12 "$OUT"/gemm_*.txt
