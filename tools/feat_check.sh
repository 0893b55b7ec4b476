# GPU check of the feature kernels: the K1-K3 parity tests (MFCC / indexing subset), then tools/feat_bench.py
# (and the MFCC phase stamps when the diagnostic build tools/_exp/libsrk_stamps.so exists)
#   gpurun --timeout 900 -- bash tools/feat_check.sh
set -o pipefail
mkdir -p gpurun_out/mf
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_features_gpu.py tests/test_indexing_gpu.py -k "${FEAT_K:-mfcc or batch}" > gpurun_out/mf/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/mf/pytest.log; grep -E "^E |FAILED" gpurun_out/mf/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/feat_bench.py 65536 || exit $?
if [ -f tools/_exp/libsrk_stamps.so ]; then
  SRK_LIB=tools/_exp/libsrk_stamps.so timeout -k 10 120 python tools/mfcc_stamps.py 65536
fi
