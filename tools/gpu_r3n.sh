#!/usr/bin/env bash
# t16 backward A/B (GWN_GCN_POW_BWD=1) with a kernel trace, then the PMC passes (metr + pems)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
rm -rf $O/prof_pb && GWN_GCN_POW_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pb -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_pb.json 2> $O/prof_pb.err || exit 1
python -c "import json; d=json.load(open('$O/prof_pb.json')); print('powbwd', d['value'], d['ms_per_step'])"
bash tools/gpu_pmc_r3.sh pmc_r3
