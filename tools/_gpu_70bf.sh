set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/pytest_fp8.log; exit 1; }
tail -1 gpurun_out/pytest_fp8.log
timeout -k 10 900 python -u bench.py --model llama3-70b --quantization fp8 --concurrency 64 --steps 200 --warmup 50 > gpurun_out/b70_fp8.json 2> gpurun_out/b70_fp8.err || { echo B70F_FAIL; tail -20 gpurun_out/b70_fp8.err; exit 1; }
cat gpurun_out/b70_fp8.json
