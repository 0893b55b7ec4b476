set -o pipefail
mkdir -p gpurun_out/g6
export TMPDIR=/tmp
PREC=bf16 timeout -k 10 120 python tools/gru_trace.py > gpurun_out/g6/trace_bf16.txt 2>&1 && tail -1 gpurun_out/g6/trace_bf16.txt
