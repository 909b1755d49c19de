#!/bin/bash
# scratch GPU command (one gpurun call): GPU suite + smoke + headline bench on the final tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/b_final.json 2> gpurun_out/b_final.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_final.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'])"
