mkdir -p gpurun_out
timeout -k 10 600 python tools/input_bench.py > gpurun_out/input_bench.json 2> gpurun_out/input_bench.err; tail -3 gpurun_out/input_bench.err; cat gpurun_out/input_bench.json
