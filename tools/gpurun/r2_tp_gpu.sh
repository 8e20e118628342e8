set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r2_tp_gpu.log 2>&1
rc=$?; echo "tp gpu rc=$rc"; tail -30 gpurun_out/r2_tp_gpu.log; exit $rc
