#!/bin/bash
# scratch GPU command (one gpurun call): GPU suite, bench x3, kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
for rep in 1 2 3; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/b_$rep.json 2>gpurun_out/b.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_$rep.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'])"
done
rm -rf gpurun_out/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
