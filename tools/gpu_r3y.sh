#!/usr/bin/env bash
# support square + tile copies in one launch: kernel tests, full GPU suite + smoke, metr + pems benches, metr kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3y}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "support_square_g4 or gram_g4" --timeout 120 --timeout-method thread > $O/t_g4.log 2>&1 || { tail -30 $O/t_g4.log; exit 1; }
tail -1 $O/t_g4.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { tail -30 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
show() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('mae12_delta'))" $1 $2; }
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_metr.json 2> $O/bench_metr.err && show $O/bench_metr.json metr &&
timeout -k 10 400 python -u bench.py --config pems --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pems.json 2> $O/bench_pems.err && show $O/bench_pems.json pems || exit 1
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || exit 1
python tools/step_trace.py $O/prof/run_kernel_trace.csv > $O/step_trace.txt; head -3 $O/step_trace.txt; grep -c . $O/step_trace.txt; grep "support" $O/step_trace.txt
