set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
DX_ASYNC_SCHEDULE=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_host_tier.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu_async.log 2>&1
rc=$?; echo "pytest async rc=$rc"; tail -3 gpurun_out/r2_pytest_gpu_async.log; [ $rc -eq 0 ] || exit $rc
for mode in 0 1 0 1; do
  DX_ASYNC_SCHEDULE=$mode timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench_async$mode.json 2> gpurun_out/r2_bench_async$mode.err
  rc=$?; echo "bench async=$mode rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/r2_bench_async$mode.json'));print(d['value'], d['ttft_p50_ms'], d['itl_p50_ms'])")"; [ $rc -eq 0 ] || exit $rc
done
