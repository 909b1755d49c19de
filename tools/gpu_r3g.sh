#!/usr/bin/env bash
# t16 cut experiments (timing only): which part of the per-tile work costs what
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
P="timeout -k 10 120 python -u tools/gcn_probe.py --ts 12,3 --reps 20"
$P --tag base 2>&1 | grep -v amdgpu.ids || exit 1
for v in ${EXPS:-nozst nores ntplain noepi}; do
GWN_LIB=graph-wavenet_amd/gwn_amd/exp/libgwn_$v.so $P --tag $v 2>&1 | grep -v amdgpu.ids || exit 1
done
