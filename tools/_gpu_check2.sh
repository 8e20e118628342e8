set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 20 600 python -u tools/router_bench.py --workers 2 --num-gpu-blocks 384 --groups 16 --prefix-len 2048 --isl 2304 --osl 16 --concurrency 16 --requests-per-conc 10 --out gpurun_out/router_bench.json > gpurun_out/router_bench.log 2>&1 || { echo ROUTER_FAIL; tail -30 gpurun_out/router_bench.log; exit 1; }
tail -1 gpurun_out/router_bench.log
