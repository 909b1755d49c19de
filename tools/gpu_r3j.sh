#!/usr/bin/env bash
# bench lines of the three configs (short) after the graph-timed roofline
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
for c in metr pems n2048; do
  st=20; [ $c = n2048 ] && st=3
  timeout -k 10 400 python -u bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline > $O/b_$c.json 2> $O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['avg_launch_us'], r['achieved'], r['frac'])"
done
