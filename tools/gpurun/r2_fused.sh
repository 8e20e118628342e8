set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --m 512 1024 2048 --rounds 3 > gpurun_out/gemm_bench_small.json 2> gpurun_out/gemm_bench_small.err
rc=$?; grep gate_up gpurun_out/gemm_bench_small.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --trace-steps > gpurun_out/r2_bench_fused.json 2> gpurun_out/r2_bench_fused.err
echo "bench rc=$?"; tail -1 gpurun_out/r2_bench_fused.json
