#!/usr/bin/env bash
# exact-vmcnt diffusion loop: kernel parity, probe, bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/gcn_probe.py --ts 12,7,3,1 --reps 20 --tag new 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print('metr', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['mae12_delta'])"
