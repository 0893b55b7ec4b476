#!/bin/bash
# Round-4 closing call 2: A/B set 11 (+ kernel census), then the PMC traffic pass.
bash tools/gpu_r04_ab11.sh r04ab11
rc=$?
echo "ab11 exit $rc"
if [ $rc -ge 2 ]; then exit $rc; fi
bash tools/gpu_round4_pmc.sh ${1:-r04g}
