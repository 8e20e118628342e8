#!/bin/bash
# the GC abort in test_chunked_mixed_matches_prefill_first reproduces only with the whole suite
# collected: same collection (tests -m gpu), engine tests only; HIP errors + C++ stacks to the log
set -o pipefail
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1 TORCH_SHOW_CPP_STACKTRACES=1 AMD_LOG_LEVEL=1 DX_GPU_TIMING=${DX_GPU_TIMING:-1}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "test_engine_gpu" > gpurun_out/engine_suitectx.log 2>&1 || { echo "FAILED rc=$?"; grep -v "^  File" gpurun_out/engine_suitectx.log | tail -30; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/engine_suitectx.log | tail -8
