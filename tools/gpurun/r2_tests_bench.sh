set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1
echo "pytest rc=$?"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --trace-steps > gpurun_out/r2_bench1.json 2> gpurun_out/r2_bench1.err
echo "bench rc=$?"
tail -1 gpurun_out/r2_bench1.json
