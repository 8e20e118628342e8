#!/bin/bash
# custom all-reduce / TP GPU tests (wall-clock barrier timeout build), then the 70B-shape TP2 rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "allreduce or tp2" > gpurun_out/ar_tests.log 2>&1 || { echo "AR TESTS FAILED"; tail -30 gpurun_out/ar_tests.log; exit 1; }
tail -2 gpurun_out/ar_tests.log
bash tools/gpurun/archive/r3_tp_rehearsal_70b.sh
