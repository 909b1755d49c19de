mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest19.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config pems --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b19_pems.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --dtype bf16 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b19_metr_bf16.json 2>/dev/null || exit 1
