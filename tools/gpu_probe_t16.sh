#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.." 2>/dev/null || cd /root/repo
for v in base l1sup nomlp nodiff; do
  if [ $v = base ]; then L=""; else L="graph-wavenet_amd/gwn_amd/exp/libgwn_$v.so"; fi
  GWN_LIB=$L timeout -k 10 120 python -u tools/gcn_probe.py --ts 12,7,3 --reps 20 --tag $v || exit 1
done
