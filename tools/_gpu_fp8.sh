set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/pytest_fp8.log; exit 1; }
tail -1 gpurun_out/pytest_fp8.log
timeout -k 10 600 python -u bench.py --quantization fp8 > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err && cat gpurun_out/bench_fp8.json || { tail -20 gpurun_out/bench_fp8.err; exit 1; }
