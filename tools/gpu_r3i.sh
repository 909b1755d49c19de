#!/usr/bin/env bash
# kernel parity (t16 paths) + probe
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gcn or support" > $O/t.log 2>&1
rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/gcn_probe.py --ts 12,7,3,1 --reps 20 --tag new 2>&1 | grep -v amdgpu.ids
