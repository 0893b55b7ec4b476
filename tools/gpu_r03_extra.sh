#!/bin/bash
# Round-3 per-model lines beside the default bench: the other precision of each config and mfrn_bgru.
#   gpurun --timeout 900 -- bash tools/gpu_r03_extra.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
run() {   # run NAME ARGS...
  local name=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-configs --no-feature-roofline --no-lowprec "$@" \
    > $OUT/bench_$name.json 2> $OUT/bench_$name.err && echo "$name $(python -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); print(d['value'], d['ms_per_step'])")"
}
run cfg3_bf16 --model fbanks_cnn --precision bf16 --steps 10 \
&& run cfg4_bf16 --model resnet_bgru --precision bf16 --steps 6 \
&& run cfg5_fp32 --model spec_bgru --precision fp32 --steps 10 \
&& run cfg5_bf16 --model spec_bgru --precision bf16 --steps 20 \
&& run mfrn_fp32 --model mfrn_bgru --precision fp32 --steps 6 \
&& run mfrn_bf16 --model mfrn_bgru --precision bf16 --steps 10
echo "exit $?"
