set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gemm_test.log 2>&1
rc=$?; tail -25 gpurun_out/gemm_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --m ${GEMM_M:-1024 2048 3000 8192} > gpurun_out/gemm_bench.json 2> gpurun_out/gemm_bench.err
rc=$?; cat gpurun_out/gemm_bench.err | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.json; exit $rc
