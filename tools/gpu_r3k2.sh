#!/usr/bin/env bash
# bf16 16-node tile forward: kernel + bf16 model tests, pems bench with trace
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3k2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config pems --steps 20 --warmup 5 --no-cpu-baseline > $O/b_pems.json 2> $O/b_pems.err || exit 1
python -c "import json; d=json.load(open('$O/b_pems.json')); r=d['roofline']; print('pems', d['value'], d['ms_per_step'], r['avg_launch_us'], r['achieved'], r['frac'], d['mae12_delta'])"
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config pems --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
python tools/step_trace.py $O/prof/run_kernel_trace.csv | head -8
