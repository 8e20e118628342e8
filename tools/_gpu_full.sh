set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1 || { echo GPU_TESTS_FAIL; tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 500 python bench.py --concurrency 192 > gpurun_out/bench_c192.json 2> gpurun_out/bench_c192.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_c192.err; exit 1; }
cat gpurun_out/bench_c192.json
