#!/bin/bash
# pipelined prefill attention (v3): numerics for both variants, then the A/B at the headline shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -k prefill --timeout 200 --timeout-method thread > gpurun_out/attn_v3_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/attn_v3_tests.log; exit 1; }
tail -3 gpurun_out/attn_v3_tests.log
timeout -k 10 300 python -u -m tools.attn_ab > gpurun_out/attn_v3_ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/attn_v3_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_v3_ab.log | head -4
