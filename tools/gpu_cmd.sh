#!/bin/bash
# scratch GPU command (one gpurun call): BN-fold kernel tests + trace + A/B bench pairs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_model.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sub.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_fold4 -o run -- python bench.py --steps 4 --warmup 3 --no-cpu-baseline > gpurun_out/fold_prof.json 2> gpurun_out/fold_prof.err &&
for k in 1 2; do
GWN_BN_FOLD=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_f1_$k.json 2>/dev/null &&
GWN_BN_FOLD=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_f0_$k.json 2>/dev/null || exit 1
done
