#!/bin/bash
# fp8 deep-stream GEMM numerics, serialized launches (AMD_SERIALIZE_KERNEL=3: a fault names its launch), the new
# test only; then, only if it passed, the w8a8 tuning report.
set -o pipefail
mkdir -p gpurun_out/dsf8
O=gpurun_out/dsf8
DX_DSTREAM_FP8=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 240 python -u -m pytest tests/test_fp8.py -m gpu -x -v -k dstream_fp8 \
  --timeout 120 --timeout-method thread > $O/tests2.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests2.log; exit 1; }
tail -8 $O/tests2.log
DX_DSTREAM_FP8=1 timeout -k 10 400 python -m tools.tune_report --fp8 --sizes 1,8,16,32,64,96,128,192,256 --out $O/tune_8b.json \
  > $O/tune_8b.log 2>&1 || { echo "TUNE FAILED"; tail -20 $O/tune_8b.log; exit 1; }
tail -40 $O/tune_8b.log
