set -o pipefail
O=gpurun_out/r01k; mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1; rc=$?
tail -30 $O/pytest.txt | grep -v "^\s*$" | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model fbanks_cnn --steps 10 --no-cpu-baseline > $O/bench_fb.json 2>$O/bench_fb.err && cat $O/bench_fb.json
