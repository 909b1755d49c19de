#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { tail -40 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
for v in 1 0 b; do
GWN_GCN_POW=${v/b/1} GWN_GCN_POW_BWD=$([ $v = b ] && echo 0 || echo 1) timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
python -c "import json; d=json.load(open('$O/bench_$v.json')); print('pow=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
done
timeout -k 10 300 python -u bench.py --config pems --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pems.json 2> $O/bench_pems.err || exit 1
python -c "import json; d=json.load(open('$O/bench_pems.json')); print('pems', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo done
