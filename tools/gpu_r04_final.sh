#!/bin/bash
# Round-4 closing call: A/B set 8 (fused dW_hh + forward worker tests, cfg2 bf16 A/B), then the evidence
# run (tools/gpu_round4.sh: pytest -m gpu, smoke, the default bench line, rocprofv3 stats per config).
# A test failure in A/B 8 (pytest exit 1) does not stop the evidence run; a timeout or crash does.
set -o pipefail
bash tools/gpu_r04_ab8.sh r04ab8
rc=$?
echo "ab8 exit $rc"
if [ $rc -ge 2 ]; then exit $rc; fi
bash tools/gpu_round4.sh ${1:-r04f}
