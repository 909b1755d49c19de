set -o pipefail
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O; shift
VAR=$1; shift
b() {
  timeout -k 10 300 env $VAR=$2 python -u bench.py --config $1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_$1_$2_$3.json 2> $O/bench_$1_$2_$3.err || { tail -20 $O/bench_$1_$2_$3.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_$1_$2_$3.json "$1 $VAR=$2 #$3"
}
for cfg in "$@"; do
  b $cfg 1 a && b $cfg 0 a && b $cfg 1 b && b $cfg 0 b && b $cfg 1 c && b $cfg 0 c || exit 1
done
