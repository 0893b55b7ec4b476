mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_evaluation_gpu.py tests/test_models_gpu.py -q -x -m gpu > gpurun_out/t.log 2>&1; tail -5 gpurun_out/t.log
