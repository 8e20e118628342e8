set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/t_gpu.log 2>&1; tail -3 gpurun_out/t_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
