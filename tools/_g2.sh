mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py tests/test_models_gpu.py -q -x -m gpu > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
timeout -k 10 300 python bench.py --model spec_cnn --steps 20 --warmup 3 --cpu-seconds 8 2>&1 | grep -v amdgpu | tail -1 > gpurun_out/b_spec_cnn.json &&
timeout -k 10 400 python bench.py --model cnn_bgru --steps 5 --warmup 2 --cpu-seconds 8 2>&1 | grep -v amdgpu | tail -1 > gpurun_out/b_cnn_bgru.json
