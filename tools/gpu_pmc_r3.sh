#!/usr/bin/env bash
# PMC passes (separate --pmc runs) over the default metr bench and the pems bf16 bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r3}
mkdir -p $O
declare -A G
G[fetch]="FETCH_SIZE"
G[write]="WRITE_SIZE"
G[sq]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
G[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_MFMA"
for cfg in metr pems; do
  for p in sq lds fetch write; do
    rm -rf $O/$cfg/$p && mkdir -p $O/$cfg
    timeout -s KILL 240 rocprofv3 --pmc ${G[$p]} --output-format csv -d $O/$cfg/$p -o run -- \
      python bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline > $O/$cfg/$p.log 2>&1 || { echo "pass $cfg $p failed"; tail -5 $O/$cfg/$p.log; exit 1; }
    echo "pass $cfg $p ok"
  done
done
python tools/pmc_table.py $O/metr/sq $O/metr/lds $O/metr/fetch $O/metr/write --match gcn_ > $O/metr_table.txt
python tools/pmc_table.py $O/pems/sq $O/pems/lds $O/pems/fetch $O/pems/write --match gcn_ > $O/pems_table.txt
python tools/pmc_summary.py $O/metr $O/pmc_bench_metr.json gcn_fwd_t16_kernel gcn_bwd_t16_kernel gram_kernel wgrad_kernel rowgemm_kernel gemm_nt_kernel > $O/metr_summary.txt
python tools/pmc_summary.py $O/pems $O/pmc_bench_pems.json gcn_fwd_t16b_kernel gcn_bwd_t16_kernel gram_g4_kernel wgrad_kernel > $O/pems_summary.txt
cp $O/pmc_bench_metr.json $O/pmc_bench_pems.json profiles/r03/  # read by the benches that follow in the same call
head -60 $O/metr_table.txt
