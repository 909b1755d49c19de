#!/bin/bash
# scratch GPU command (one gpurun call): balanced-layout parity + micro-bench, prefetch 3 vs 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layouts_agree or per_sample_supports" > gpurun_out/t_bal.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_gcn.py --reps 20 > gpurun_out/bench_gcn_bal3.log 2>&1 &&
GWN_LIB=$PWD/graph-wavenet_amd/gwn_amd/exp/libgwn_pf2.so timeout -k 10 200 python -u tools/bench_gcn.py --reps 20 > gpurun_out/bench_gcn_bal2.log 2>&1
