#!/bin/bash
# custom-AR / TP GPU tests (reported, not gating), 70B-shape TP2 rehearsal, then the HTTP / serving-graph benchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "allreduce or tp2" > gpurun_out/ar_tests.log 2>&1; RC=$?
tail -3 gpurun_out/ar_tests.log
grep -n "AssertionError" gpurun_out/ar_tests.log
case $RC in 0|1) ;; *) echo "AR tests ended with $RC: stopping"; exit $RC;; esac
bash tools/gpurun/archive/r3_tp_rehearsal_70b.sh || exit 1
bash tools/gpurun/archive/r3_http.sh
