#!/bin/bash
# Round-4: per-step phase timeline of the 16-bit backward recurrence with and without the fused dW_hh
# worker waves (tools/gru_trace.py, layer-1 shape of cfg2: B = 256, T = 51, in = 1024).
set -o pipefail
OUT=gpurun_out/${1:-r04trace}
mkdir -p "$OUT"
for dw in 0 1; do
  PREC=bf16 SRK_OPTIONS=gru_dwhh_fused=$dw timeout -k 10 120 python tools/gru_trace.py > "$OUT/trace_bf16_dw$dw.txt" 2>&1 || exit $?
done
tail -n 20 "$OUT"/trace_bf16_dw*.txt
