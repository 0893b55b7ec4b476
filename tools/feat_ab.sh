#!/bin/bash
# A/B timing of feature-kernel variants built by tools/build_variant.sh (tools/_exp/libsrk_NAME.so):
#   gpurun -- bash tools/feat_ab.sh NAME1 NAME2 ...   (FEAT_ONLY=mfcc,... selects kernels; "main" = the in-tree build)
# Each variant first runs the K1-K3 parity tests (FEAT_K selects a subset), so a wrong variant is not timed.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = main ]; then lib=speechrecognitionproject_amd/libsrk.so; else lib=tools/_exp/libsrk_$v.so; fi
  SRK_LIB=$lib timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_features_gpu.py tests/test_indexing_gpu.py ${FEAT_K:+-k "$FEAT_K"} > gpurun_out/ab/pytest_$v.log 2>&1 \
    || { echo "$v: parity FAILED"; grep -E "^E |FAILED" gpurun_out/ab/pytest_$v.log | head -20; exit 1; }
  echo "$v: parity ok; $(SRK_LIB=$lib timeout -k 10 120 python tools/feat_bench.py 65536)" || exit 1
done
