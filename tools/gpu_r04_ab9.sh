#!/bin/bash
# Round-4 A/B set 9: BatchNorm-emitted 16-bit conv operands (parity, then cfg4 / mfrn bf16 with and without).
set -o pipefail
OUT=gpurun_out/${1:-r04ab9}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_copy16_gpu.py \
  > "$OUT/pytest_bn16.log" 2>&1 || { rc=$?; tail -40 "$OUT/pytest_bn16.log"; exit $rc; }
tail -3 "$OUT/pytest_bn16.log"
run() {  # run TAG BN_COPY16 ARGS...
  local tag=$1 on=$2; shift 2
  SRK_BN_COPY16=$on timeout -k 10 300 python bench.py --no-lowprec --no-cpu-baseline --no-feature-roofline "$@" \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
}
run cfg4_bf16_bn0 0 --model resnet_bgru --precision bf16 --batch 512 --steps 5
run cfg4_bf16_bn1 1 --model resnet_bgru --precision bf16 --batch 512 --steps 5
run mfrn_bf16_bn0 0 --model mfrn_bgru --precision bf16 --steps 10
run mfrn_bf16_bn1 1 --model mfrn_bgru --precision bf16 --steps 10
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), r["value"], r["ms_per_step"], {k: round(v["ms_total"], 3) for k, v in r["kernels"].items()})
PY
