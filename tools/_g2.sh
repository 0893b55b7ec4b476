set -o pipefail
O=gpurun_out/r01c; mkdir -p $O
timeout -k 10 120 python tools/gemm_bench.py > $O/gemm.txt 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_dense_gpu.py tests/test_models_gpu.py tests/test_conv_gpu.py tests/test_training_gpu.py -x -q > $O/pytest.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfcc-roofline > $O/bench.json 2>$O/bench.err
rc=$?; grep -v "^{" $O/gemm.txt; tail -2 $O/pytest.txt; cat $O/bench.json; exit $rc
