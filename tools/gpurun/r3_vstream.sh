#!/bin/bash
# register-streamed decode GEMM: numerics tests, then the shape sweep vs hipBLASLt and the older kernels
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_skinny_gemm.py -m gpu -x -v -k vstream --timeout 200 --timeout-method thread > gpurun_out/vstream_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/vstream_tests.log; exit 1; }
tail -3 gpurun_out/vstream_tests.log
timeout -k 10 600 python -u -m tools.vstream_bench --out gpurun_out/vstream.json ${VS_ARGS:---old} > gpurun_out/vstream_bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/vstream_bench.log; exit 1; }
cat gpurun_out/vstream_bench.log
