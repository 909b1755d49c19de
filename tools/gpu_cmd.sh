#!/bin/bash
# scratch GPU command (one gpurun call): rehearse bench.py's N=2 data-parallel path on one GPU (gloo)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GWN_DIST_BACKEND=gloo GWN_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/b_n2.json 2> gpurun_out/b_n2.err || { tail -30 gpurun_out/b_n2.err; exit 1; }
cat gpurun_out/b_n2.json
