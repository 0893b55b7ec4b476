set -o pipefail
O=gpurun_out/v1
mkdir -p $O
export TMPDIR=/tmp
summ() { python - "$1" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1])); b = d.get("bf16", {})
print(sys.argv[1], "fp32", d["value"], d["ms_per_step"], {k: v["ms_total"] for k, v in d["kernels"].items()})
print("   bf16", b.get("value"), b.get("ms_per_step"), {k: v["ms_total"] for k, v in b.get("kernels", {}).items()})
EOF
}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert|^E ' $O/pytest.log | head -30; exit $rc; }
for c in 3 4; do
  SRK_H16_CFG=$c timeout -k 10 150 python tools/gemm_bench.py --precision bf16 --h16 > $O/gemm_h16_cfg$c.txt 2>&1 || exit 1
  echo "cfg $c"; grep -v '^{' $O/gemm_h16_cfg$c.txt
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-feature-roofline > $O/bench.json 2> $O/bench.err || exit 1
summ $O/bench.json
for m in fbanks_cnn resnet_bgru; do
  timeout -k 10 400 python bench.py --model $m --steps 10 --no-cpu-baseline --no-feature-roofline > $O/bench_$m.json 2> $O/bench_$m.err || exit 1
  summ $O/bench_$m.json
done
