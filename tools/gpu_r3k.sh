#!/usr/bin/env bash
# GPU tests, the trajectory test's numbers, default bench lines (metr, pems) and a kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1
rc=$?
# 1 = assertion failures only (keep measuring); anything else (crash, fault, time limit) ends the call
[ $rc -le 1 ] || { tail -40 $O/t_all.log; exit 1; }
grep -E "^(FAILED|ERROR)|passed|failed" $O/t_all.log || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -q -s -k tracks_fp32 --timeout 250 --timeout-method thread > $O/t_traj.log 2>&1
[ $? -le 1 ] || exit 1
grep "loss fp32" $O/t_traj.log || true
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print('metr', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
timeout -k 10 300 python -u bench.py --config pems --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pems.json 2> $O/bench_pems.err || exit 1
python -c "import json; d=json.load(open('$O/bench_pems.json')); print('pems', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo done
