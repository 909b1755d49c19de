#!/usr/bin/env bash
# round 3, first GPU check of the power-schedule GCN kernels: kernel + model + headline tests,
# then the full GPU suite, smoke, and a bench line each for the power and the chained schedule
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "square or schedules or split_many or pow_forward or per_sample" > $O/t_kern.log 2>&1 || { tail -40 $O/t_kern.log; exit 1; }
tail -3 $O/t_kern.log
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { tail -40 $O/t_all.log; exit 1; }
tail -3 $O/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_pow.json 2> $O/bench_pow.err || exit 1
GWN_GCN_POW=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_chain.json 2> $O/bench_chain.err || exit 1
python - <<'PY'
import json
for k in ("pow", "chain"):
    d = json.load(open("gpurun_out/r3a/bench_%s.json" % k))
    print(k, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"], d["mae12_delta"])
PY
rm -rf $O/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo done
