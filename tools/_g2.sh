set -o pipefail
O=gpurun_out/r01f; mkdir -p $O
timeout -k 10 120 python tools/gru_trace.py > $O/trace.txt 2>&1; rc=$?
cat $O/trace.txt | grep -v amdgpu.ids; exit $rc
