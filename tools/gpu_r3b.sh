#!/usr/bin/env bash
# round 3: what bounds the power-schedule GCN kernels (probe variants + PMC)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
P="timeout -k 10 120 python -u tools/gcn_probe.py --reps 20"
$P --tag pow > $O/probe.txt 2>&1 &&
$P --tag chain --chain >> $O/probe.txt 2>&1 &&
$P --tag nopieces --no-pieces >> $O/probe.txt 2>&1 &&
GWN_LIB=graph-wavenet_amd/gwn_amd/exp/libgwn_noG.so $P --tag noG >> $O/probe.txt 2>&1 &&
GWN_LIB=graph-wavenet_amd/gwn_amd/exp/libgwn_noLDS.so $P --tag noLDS >> $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
for p in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
         "TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr" ; do
  tag=$(echo $p | cut -c1-12 | tr ' ' '_')
  rm -rf $O/pmc_$tag
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $O/pmc_$tag -o run -- python tools/gcn_probe.py --reps 3 --ts 12 > $O/pmc_$tag.log 2>&1 || echo "pmc pass $tag failed"
done
echo done
