#!/bin/bash
# isolate the GC abort seen in test_chunked_mixed_matches_prefill_first: engine tests without, then
# with, the per-launch timing events; every GPU step under its own limit, stop at the first failure
set -o pipefail
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
DX_GPU_TIMING=0 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/engine_notiming.log 2>&1 || { echo "notiming FAILED"; grep -E "PASSED|FAILED|Error|Abort" gpurun_out/engine_notiming.log | tail -12; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/engine_notiming.log | tail -8
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/engine_timing.log 2>&1 || { echo "timing FAILED"; grep -E "PASSED|FAILED|Error|Abort" gpurun_out/engine_timing.log | tail -12; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/engine_timing.log | tail -8
