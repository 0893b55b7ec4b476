mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
