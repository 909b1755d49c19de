mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for ov in ${OVS:-1 0}; do
GWN_OVERLAP=$ov timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ov$ov.json 2>gpurun_out/bench_ov$ov.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_ov$ov.json'));print('overlap',$ov,d['value'],d['ms_per_step'])"
done
rm -rf gpurun_out/prof
GWN_OVERLAP=${PROF_OVERLAP:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
