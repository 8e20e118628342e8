#!/bin/bash
# 3/6/7-wave dstream configs: numerics, then the driver's bench command with the decode-GEMM tuning table, then
# the HTTP serving A/B (tools/gpurun/r5_http_ab.sh) on the same box.
set -o pipefail
mkdir -p gpurun_out/r5db
O=gpurun_out/r5db
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_skinny_gemm.py -m gpu \
  -k dstream > $O/dstream_tests.txt 2>&1 || { tail -30 $O/dstream_tests.txt; exit 1; }
tail -1 $O/dstream_tests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --gemm-report $O/gemm_report.json \
  > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-220
bash tools/gpurun/r5_http_ab.sh 0.0005 0.0001
