#!/usr/bin/env bash
# full GPU suite + smoke, metr bench, kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { tail -30 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_metr.json 2> $O/bench_metr.err || exit 1
python -c "import json; d=json.load(open('$O/bench_metr.json')); print('metr', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || exit 1
python tools/step_trace.py $O/prof/run_kernel_trace.csv | head -14
