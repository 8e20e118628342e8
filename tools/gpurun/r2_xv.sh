set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/xv
timeout -k 10 300 python -u -m pytest tests/test_skinny_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xv/pytest.log 2>&1
rc=$?; echo "pytest skinny rc=$rc"; tail -3 gpurun_out/xv/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m tools.wstream_xv_probe > gpurun_out/xv/probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/xv/probe.txt | grep -v amdgpu.ids; exit $rc
