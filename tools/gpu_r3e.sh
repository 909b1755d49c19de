#!/usr/bin/env bash
# t16 kernel experiments: probe the product build in several modes and the experiment builds
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
P="timeout -k 10 120 python -u tools/gcn_probe.py --ts 12,7,3,1 --reps 20"
$P --tag base > $O/base.log 2>&1 && cat $O/base.log || exit 1
$P --tag drop0 --drop 0 > $O/drop0.log 2>&1 && cat $O/drop0.log || exit 1
$P --tag nopieces --no-pieces > $O/nop.log 2>&1 && cat $O/nop.log || exit 1
$P --tag nobn --no-bn > $O/nobn.log 2>&1 && cat $O/nobn.log || exit 1
for v in ring6 ring3 img2; do
GWN_LIB=graph-wavenet_amd/gwn_amd/exp/libgwn_$v.so $P --tag $v > $O/$v.log 2>&1 && cat $O/$v.log || exit 1
done
