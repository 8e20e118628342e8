set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_ms4.json 2> gpurun_out/bench_ms4.err && cat gpurun_out/bench_ms4.json || exit 1
DX_MULTI_STEP=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench_ms1.json 2> gpurun_out/bench_ms1.err && cat gpurun_out/bench_ms1.json || exit 1
timeout -k 10 400 python -u tools/role_bench.py --role decode > gpurun_out/roles_ms4.json 2> gpurun_out/roles_ms4.err && cat gpurun_out/roles_ms4.json
