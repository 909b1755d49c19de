set -o pipefail
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r5k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/t_all.log 2>&1 || { tail -40 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
b() {
  timeout -k 10 400 python -u bench.py --config $1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_$2.json 2> $O/bench_$2.err || { tail -20 $O/bench_$2.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('mae12_delta'))" $O/bench_$2.json $2
}
b metr metr1 && b metr metr2 && b pems pems1 && b pems pems2 || exit 1
tools/gpu.sh ${1:-r5k} stats:metr
