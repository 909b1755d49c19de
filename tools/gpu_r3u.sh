#!/usr/bin/env bash
# tiled bf16 gram: tile-block size 2 / 3 / 4 (kernel tests + pems bf16 bench each), kernel stats of the default
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3u}
mkdir -p $O
show() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('mae12_delta'))" $1 $2; }
for tb in 3 2 4; do
  GWN_GRAM_TB=$tb timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q -k "gram_g4 or bf16_train" --timeout 120 --timeout-method thread > $O/t_g4_$tb.log 2>&1 || { tail -30 $O/t_g4_$tb.log; exit 1; }
  tail -1 $O/t_g4_$tb.log
  GWN_GRAM_TB=$tb timeout -k 10 400 python -u bench.py --config pems --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pems_$tb.json 2> $O/bench_pems_$tb.err && show $O/bench_pems_$tb.json pems-tb$tb || exit 1
done
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config pems --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || exit 1
python tools/step_trace.py $O/prof/run_kernel_trace.csv > $O/step_trace.txt; head -8 $O/step_trace.txt
