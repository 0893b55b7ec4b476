set -o pipefail
O=gpurun_out/v2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model spec_bgru --precision fp16 --steps 10 --no-cpu-baseline > $O/bench_spec_bgru_fp16.json 2> $O/bench_spec_bgru_fp16.err || { tail -5 $O/bench_spec_bgru_fp16.err; exit 1; }
cut -c1-600 $O/bench_spec_bgru_fp16.json
