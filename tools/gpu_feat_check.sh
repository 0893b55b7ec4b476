#!/bin/bash
# A feature-kernel change on the GPU:  gpurun --timeout 900 -- bash tools/gpu_feat_check.sh TAG
# the feature / model tests, the feature rooflines (bench.py: K1 on 65,536 clips, K2 and K3 beside it), then the
# SQ instruction counters of K1-K3 (tools/feat_pmc.sh, SQ passes only).
set -o pipefail
TAG=${1:-feat}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_features_gpu.py tests/test_models_gpu.py tests/test_indexing_gpu.py \
  -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-h2d --no-prof --no-lowprec \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json
d = json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
for r in [d['feature_roofline']] + d.get('feature_roofline_other', []):
    print(r['kernel'], r['achieved'], 'GB/s', r['frac'], r['ms_per_launch'], 'ms')
"
[ -n "$NO_PMC" ] || { timeout -k 10 700 bash tools/feat_pmc.sh "$TAG/feat" > "$OUT/feat_pmc.log" 2>&1; rc=$?; tail -30 "$OUT/feat_pmc.log"; exit $rc; }
