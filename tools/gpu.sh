#!/usr/bin/env bash
# One parametrised GPU-box script (run through gpurun): a sequence of steps, each under its own
# time limit, stopping at the first failure.  Output under gpurun_out/<out>/.
#
#   tools/gpu.sh <out> step [step ...]
#
# steps:
#   suite                 the whole -m gpu suite, then smoke()
#   test:<file|-k expr>   pytest -m gpu on one file (tests/...py) or a -k expression
#   bench:<cfg>[:<dtype>] one bench.py line (cfg metr|pems|n2048; no CPU baseline); "default" =
#                         the driver's invocation (python bench.py, with the CPU baseline)
#   stats:<cfg>[:<dtype>] rocprofv3 kernel trace + stats of a short bench, and its one-step trace
#   pmc:<cfg>             the four PMC passes (sq, lds, fetch, write) over a short bench + summary
#   cmd:<python args>     python <args> (a probe / microbenchmark; ':' separates arguments)
#
# Env: STEPS / WARMUP for bench (default 30 / 5), EXTRA_ENV="A=1 B=2" exported before every step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for kv in ${EXTRA_ENV:-}; do export "$kv"; done
O=gpurun_out/$1
shift
mkdir -p "$O"
show() { python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], r.get('avg_launch_us'), d.get('mae12_delta'), (d.get('cpu_baseline') or {}).get('value'))" "$1" "$2"; }
kernels() {  # PMC summary kernels per config
  case $1 in
    pems) echo "gcn_fwd_t16b2_kernel gcn_fwd_t16b_kernel gcn_bwd_t16_kernel gram_cu_g4_kernel wgrad_group_kernel rowgemm_kernel gemm_nt_bf16_kernel wgrad_bf16_kernel" ;;
    *) echo "gcn_fwd_t16_kernel gcn_bwd_t16_kernel gram_cu_kernel wgrad_group_kernel rowgemm_kernel gemm_nt_kernel gemm_kernel" ;;
  esac
}
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  cfg=${arg%%:*}; dt=${arg#*:}; [ "$dt" = "$arg" ] && dt=""
  dflag=""; [ -n "$dt" ] && dflag="--dtype $dt"
  tag=${cfg}${dt:+_$dt}
  echo "== $step"
  case $kind in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { tail -30 $O/t_all.log; exit 1; }
      tail -1 $O/t_all.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      echo smoke ok ;;
    test)
      if [[ "$arg" == tests/* ]]; then sel=(${arg//,/ }); else sel=(tests -k "$arg"); fi
      log=$O/t_$(echo "$arg" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-40).log
      timeout -k 10 600 python -u -m pytest "${sel[@]}" -m gpu -x -q --timeout 120 --timeout-method thread > $log 2>&1 || { tail -40 $log; exit 1; }
      tail -1 $log ;;
    bench)
      if [ "$cfg" = "default" ]; then
        timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
        show $O/bench_default.json default || exit 1
      else
        timeout -k 10 400 python -u bench.py --config $cfg $dflag --steps ${STEPS:-30} --warmup ${WARMUP:-5} --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
        show $O/bench_$tag.json $tag || exit 1
      fi ;;
    stats)
      rm -rf $O/prof_$tag
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python bench.py --config $cfg $dflag --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$tag.json 2> $O/prof_$tag.err || { tail -20 $O/prof_$tag.err; exit 1; }
      python tools/step_trace.py $O/prof_$tag/run_kernel_trace.csv --list > $O/step_$tag.txt && head -30 $O/step_$tag.txt ;;
    pmc)
      declare -A G
      G[fetch]="FETCH_SIZE"
      G[write]="WRITE_SIZE"
      G[sq]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
      G[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_MFMA"
      for p in sq lds fetch write; do
        rm -rf $O/pmc_$tag/$p && mkdir -p $O/pmc_$tag
        timeout -s KILL 240 rocprofv3 --pmc ${G[$p]} --output-format csv -d $O/pmc_$tag/$p -o run -- \
          python bench.py --config $cfg $dflag --steps 3 --warmup 2 --no-cpu-baseline > $O/pmc_$tag/$p.log 2>&1 || { echo "pass $p failed"; tail -5 $O/pmc_$tag/$p.log; exit 1; }
        echo "pass $p ok"
      done
      python tools/pmc_summary.py $O/pmc_$tag $O/pmc_bench_$tag.json $(kernels $cfg) > $O/pmc_${tag}_summary.txt && cat $O/pmc_${tag}_summary.txt ;;
    cmd)
      timeout -k 10 300 python -u ${arg//:/ } > $O/cmd.log 2>&1 || { tail -30 $O/cmd.log; exit 1; }
      tail -40 $O/cmd.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh done"
