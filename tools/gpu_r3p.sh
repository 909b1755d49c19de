#!/usr/bin/env bash
# persistent t16 kernels: kernel + model parity, bench A/B (t16 backward on / off), kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
[ $rc -eq 0 ] || exit 1
for v in 0 1; do
GWN_GCN_POW_BWD=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_pb$v.json 2> $O/bench_pb$v.err || exit 1
python -c "import json; d=json.load(open('$O/bench_pb$v.json')); print('powbwd=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
done
rm -rf $O/prof && GWN_GCN_POW_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || exit 1
echo done
