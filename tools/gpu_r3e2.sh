#!/usr/bin/env bash
# support-fragment access experiments (timing only; wrong results): tiled layout, same columns
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3e2
mkdir -p $O
P="timeout -k 10 120 python -u tools/gcn_probe.py --ts 12,7 --reps 20"
$P --tag base > $O/base.log 2>&1 && cat $O/base.log || exit 1
for v in tiled samecol; do
GWN_LIB=graph-wavenet_amd/gwn_amd/exp/libgwn_$v.so $P --tag $v > $O/$v.log 2>&1 && cat $O/$v.log || exit 1
done
