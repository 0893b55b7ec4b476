set -o pipefail
O=gpurun_out/r01e; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_dense_gpu.py -x -q -k persistent > $O/pytest_p.txt 2>&1; rc=$?
tail -30 $O/pytest_p.txt
[ $rc -eq 0 ] && timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfcc-roofline > $O/bench.json 2>$O/bench.err
rc=$?; tail -2 $O/pytest.txt; cat $O/bench.json; tail -3 $O/bench.err; exit $rc
