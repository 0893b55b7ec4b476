set -o pipefail
O=gpurun_out/r01x; mkdir -p $O
timeout -k 10 200 python -m pytest tests/test_dense_gpu.py tests/test_models_gpu.py -q -x -k "gru or golden or model" > $O/pt.txt 2>&1; rc=$?; tail -3 $O/pt.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gru_trace.py > $O/trace.txt 2>&1 && grep -v amdgpu $O/trace.txt && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-feature-roofline > $O/bench.json 2>$O/bench.err && cat $O/bench.json
