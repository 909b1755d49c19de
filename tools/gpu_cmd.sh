#!/bin/bash
# scratch GPU command (one gpurun call): GPU suite + smoke, then the round's measurement set
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/profile_round.sh
