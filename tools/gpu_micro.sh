# GPU-box script: GCN micro-benchmark (fused forward / backward variants)
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_gcn.py --ts 12,9,4,3,1 > gpurun_out/bench_gcn.txt 2>&1; rc=$?; cat gpurun_out/bench_gcn.txt; exit $rc
