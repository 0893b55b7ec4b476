mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_augment_gpu.py -q -x -m gpu > gpurun_out/t.log 2>&1; tail -30 gpurun_out/t.log
