#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 250 --timeout-method thread > gpurun_out/tp_gpu.log 2>&1 || { echo "TP FAILED"; grep -E "PASSED|FAILED|Error" gpurun_out/tp_gpu.log | tail -20; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/tp_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
