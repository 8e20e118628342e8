set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gemm.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_skinny.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/t_skinny.log; exit 1; }
tail -3 gpurun_out/t_skinny.log
PYTHONPATH=. timeout -k 10 400 python -u tools/skinny_bench.py --out gpurun_out/skinny.json > gpurun_out/skinny.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/skinny.log; exit 1; }
cat gpurun_out/skinny.log
