set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_host_tier.py tests/test_disagg.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_host.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_pytest_host.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 900 python -u tools/multiturn_bench.py --model deepseek-r1-distill-llama-8b --users 32 --rounds 10 --first 2000 --turn 100 --osl 150 --gpu-blocks 700 --host-blocks 0,2400 --out gpurun_out/r2_multiturn.json > gpurun_out/r2_multiturn.log 2>&1
rc=$?; echo "multiturn rc=$rc"; tail -4 gpurun_out/r2_multiturn.log
