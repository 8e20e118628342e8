#!/bin/bash
# Round 6: one-sided KV transport, prefill TP1 -> decode TP2 (three processes on one GPU).
set -o pipefail
out=${1:-gpurun_out/r6_ipc_tp}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_disagg_loopback.py -m gpu -k "tp2_one_gpu_ipc" > "$out/tests.log" 2>&1
rc=$?
tail -15 "$out/tests.log"
exit $rc
