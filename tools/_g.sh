set -o pipefail
mkdir -p gpurun_out/g3
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g3/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/g3/pytest.log; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert' gpurun_out/g3/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-feature-roofline > gpurun_out/g3/bench_fp32.json 2> gpurun_out/g3/bench_fp32.err && cat gpurun_out/g3/bench_fp32.json && \
timeout -k 10 200 python bench.py --precision bf16 --no-cpu-baseline --no-feature-roofline > gpurun_out/g3/bench_bf16.json 2> gpurun_out/g3/bench_bf16.err && cat gpurun_out/g3/bench_bf16.json
