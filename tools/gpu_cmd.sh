#!/bin/bash
# scratch GPU command (one gpurun call): gram-first order A/B + trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_model.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sub.log 2>&1 &&
for k in 1 2 3; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_g_$k.json 2>/dev/null || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gfirst -o run -- python bench.py --steps 4 --warmup 3 --no-cpu-baseline > gpurun_out/gf_prof.json 2> gpurun_out/gf_prof.err
