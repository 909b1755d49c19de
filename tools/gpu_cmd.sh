#!/bin/bash
# scratch GPU command (one gpurun call): deferred wgrad reduction: suite + A/B + trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 &&
for k in 1 2; do
GWN_DEFER_WGRAD=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_d1_$k.json 2>/dev/null &&
GWN_DEFER_WGRAD=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/ab_d0_$k.json 2>/dev/null || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_defer -o run -- python bench.py --steps 4 --warmup 3 --no-cpu-baseline > gpurun_out/defer_prof.json 2> gpurun_out/defer_prof.err
