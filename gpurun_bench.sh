#!/usr/bin/env bash
# GPU-box script: bench (JSON line) + rocprofv3 kernel-trace stats of a short bench run.
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps ${STEPS:-30} --warmup ${WARMUP:-5} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || exit $?
fi
