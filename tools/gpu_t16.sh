#!/usr/bin/env bash
# the 16-node tile forward: kernel parity tests, then bench A/B against the 32-node tiles
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-t16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || exit 1
for v in 10 11 00; do
GWN_GCN_T16=${v:0:1} GWN_GCN_POW_BWD=${v:1:1} timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
python -c "import json; d=json.load(open('$O/bench_$v.json')); print('t16,powbwd=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
done
GWN_GCN_T16=1 timeout -k 10 300 python -u bench.py --config pems --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pems.json 2> $O/bench_pems.err || exit 1
python -c "import json; d=json.load(open('$O/bench_pems.json')); print('pems', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
rm -rf $O/prof && GWN_GCN_POW_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo done
