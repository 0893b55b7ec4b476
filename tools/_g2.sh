set -o pipefail
O=gpurun_out/r01z; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_dense_gpu.py tests/test_models_gpu.py tests/test_training_gpu.py -q -x > $O/pt.txt 2>&1; rc=$?; tail -2 $O/pt.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gemm_bench.py > $O/gemm.txt 2>&1 && grep -v "amdgpu\|^{" $O/gemm.txt && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-feature-roofline > $O/bench.json 2>$O/bench.err && cat $O/bench.json
