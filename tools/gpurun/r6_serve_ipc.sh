#!/bin/bash
# Round 6: the served disaggregated graph with the one-sided (ipc) KV transport on one GPU.
set -o pipefail
out=${1:-gpurun_out/r6_serve_ipc}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread \
  tests/test_serve_disagg_gpu.py -m gpu -k one_sided > "$out/tests.log" 2>&1
rc=$?
tail -15 "$out/tests.log"
exit $rc
