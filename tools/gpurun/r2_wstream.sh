set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_skinny_gemm.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ws_test.log 2>&1
rc=$?; tail -15 gpurun_out/ws_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m tools.skinny_bench --ms ${WS_M:-64,128,256} --out gpurun_out/ws_bench.json > gpurun_out/ws_bench.log 2>&1
rc=$?; cat gpurun_out/ws_bench.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m tools.wstream_probe > gpurun_out/probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/probe.log; exit $rc
