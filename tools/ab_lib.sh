# Same-box A/B of the product library against an experiment build (tools/exp_build.sh):
#   bash tools/ab_lib.sh <out> <exp name> <cfgs...>   (runs through gpurun; prints value, ms/step)
set -o pipefail
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O; shift
X=$1; shift
b() {  # cfg lib(product|exp) rep
  local lib=""; [ "$2" = exp ] && lib=graph-wavenet_amd/gwn_amd/exp/libgwn_$X.so
  timeout -k 10 300 env GWN_LIB=$lib python -u bench.py --config $1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_$1_$2_$3.json 2> $O/bench_$1_$2_$3.err || { tail -20 $O/bench_$1_$2_$3.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" $O/bench_$1_$2_$3.json "$1 $2 #$3"
}
for cfg in "$@"; do
  b $cfg product a && b $cfg exp a && b $cfg product b && b $cfg exp b && b $cfg product c && b $cfg exp c || exit 1
done
