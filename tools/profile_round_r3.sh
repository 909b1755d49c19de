#!/usr/bin/env bash
# GPU-box script: round-3 measurement set -> gpurun_out/round3/
#   GPU suite + smoke, bench lines (metr headline with CPU baseline, pems bf16 / fp32, n2048),
#   rocprofv3 kernel stats of the metr and pems benches
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/round3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { tail -30 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
echo "bench metr" && timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > $O/bench_metr.json 2> $O/bench_metr.err &&
echo "bench pems bf16" && timeout -k 10 400 python -u bench.py --config pems --steps 20 --warmup 5 > $O/bench_pems_bf16.json 2> $O/bench_pems_bf16.err &&
echo "bench pems f32" && timeout -k 10 300 python -u bench.py --config pems --dtype f32 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pems_f32.json 2> $O/bench_pems_f32.err &&
echo "bench n2048" && timeout -k 10 500 python -u bench.py --config n2048 --steps 5 --warmup 2 > $O/bench_n2048.json 2> $O/bench_n2048.err &&
echo "stats metr" && rm -rf $O/prof_metr && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_metr -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_metr.json 2> $O/prof_metr.err &&
echo "stats pems" && rm -rf $O/prof_pems && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pems -o run -- python bench.py --config pems --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_pems.json 2> $O/prof_pems.err &&
for f in metr pems_bf16 pems_f32 n2048; do python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'), d.get('mae12_delta'))"; done &&
echo "round measurements done"
