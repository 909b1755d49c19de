#!/bin/bash
# scratch GPU command (one gpurun call): gram-on-side-stream mode -- model tests with it on, A/B bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GWN_GRAM_SIDE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ddp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_side.log 2>&1 || { tail -30 gpurun_out/t_side.log; exit 1; }
tail -2 gpurun_out/t_side.log
for rep in 1 2; do
for gs in 0 1; do
GWN_GRAM_SIDE=$gs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/gs_${gs}_$rep.json 2>gpurun_out/gs.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/gs_${gs}_$rep.json'));print('gram_side',$gs,d['value'],d['ms_per_step'])"
done
done
GWN_GRAM_SIDE=1 timeout -k 10 200 python bench.py --config pems --no-cpu-baseline --steps 20 > gpurun_out/gs_pems.json 2>gpurun_out/gs.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/gs_pems.json'));print('pems gram_side',d['value'],d['ms_per_step'])"
