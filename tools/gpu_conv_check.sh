#!/bin/bash
# One conv change on the GPU:  gpurun --timeout 900 -- bash tools/gpu_conv_check.sh TAG "test files" ["-k expression"]
# the selected tests, then rocprofv3 kernel stats of the cfg3 fp32 and bf16 bench commands (graph replays);
# AB_OPTS="opt=v,...": a third cfg3 fp32 run with those srk options (SRK_OPTIONS).
set -o pipefail
TAG=${1:-conv}
SEL=${2:-tests/test_conv_gpu.py}
KEXPR=${3:-gpu}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
stats() {   # stats NAME ARGS...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/stats_${name}" -o run -- \
    python3 bench.py --no-cpu-baseline --no-configs --no-feature-roofline --no-h2d "$@" \
    > "$OUT/stats_${name}.json" 2> "$OUT/stats_${name}.err" \
  && python3 tools/rocpd_summary.py "$OUT/stats_${name}" > "$OUT/summary_${name}_stats.txt" && rm -rf "$OUT/stats_${name}"
}
timeout -k 10 600 python -u -m pytest $SEL -k "$KEXPR" -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || exit $rc
stats cfg3 --model fbanks_cnn --no-lowprec --steps 10 && echo "cfg3: $(tail -c 300 $OUT/stats_cfg3.json | head -c 200)" \
  && stats cfg3b --model fbanks_cnn --precision bf16 --no-lowprec --steps 10 \
  && { [ -z "$AB_OPTS" ] || SRK_OPTIONS="$AB_OPTS" stats cfg3ab --model fbanks_cnn --no-lowprec --steps 10; } && echo "stats ok"
