#!/usr/bin/env bash
# GPU-box script: PMC counter passes (one counter group per rocprofv3 run, --pmc only, no traces)
# over a command, default the GCN micro-benchmark.  Output: gpurun_out/pmc/<pass>/run_counter_collection.csv
#   PASSES="fetch write sq lds" tools/pmc.sh [python args...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tools/bench_gcn.py --reps 5 --ts 12)
declare -A GROUPS_
GROUPS_[fetch]="FETCH_SIZE"
GROUPS_[write]="WRITE_SIZE"
GROUPS_[sq]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
GROUPS_[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_MFMA"
GROUPS_[l2]="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
for p in ${PASSES:-fetch write sq lds}; do
  rm -rf gpurun_out/pmc/$p
  timeout -k 10 300 rocprofv3 --pmc ${GROUPS_[$p]} --output-format csv -d gpurun_out/pmc/$p -o run -- \
    python "${ARGS[@]}" > gpurun_out/pmc/$p.log 2>&1 || { echo "pass $p failed"; tail -20 gpurun_out/pmc/$p.log; exit 1; }
done
echo "pmc passes done"
