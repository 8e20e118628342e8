set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/mb_attn.json 2> gpurun_out/mb_attn.err && timeout -k 10 300 python tools/microbench.py --what decode > gpurun_out/mb_dec.json 2> gpurun_out/mb_dec.err && cat gpurun_out/mb_attn.json gpurun_out/mb_dec.json | tr -d '\n '
echo
timeout -k 10 600 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err && cat gpurun_out/bench_n1.json
timeout -k 10 600 python -u tools/role_bench.py --role decode > gpurun_out/roles.json 2> gpurun_out/roles.err && cat gpurun_out/roles.json
