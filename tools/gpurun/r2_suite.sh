set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu_head.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_pytest_gpu_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke_head.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r2_smoke_head.log; exit $rc
