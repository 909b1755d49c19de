#!/bin/bash
# scratch GPU command (one gpurun call): double-buffered LDS gram parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gram" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gram.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_gcn.py --reps 20 > gpurun_out/bench_gcn_gram.log 2>&1
