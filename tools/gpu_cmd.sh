#!/bin/bash
# scratch GPU command (one gpurun call): GPU suite, split A/B, then the round's measurement set
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
for rep in 1 2; do
for thr in 0 default; do
if [ $thr = default ]; then unset GWN_KSPLIT_SLICES; else export GWN_KSPLIT_SLICES=$thr; fi
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/ks_${thr}_$rep.json 2>gpurun_out/ks_${thr}.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/ks_${thr}_$rep.json'));print('thr','$thr',d['value'],d['ms_per_step'])"
done
done
unset GWN_KSPLIT_SLICES
bash tools/profile_round.sh
