#!/bin/bash
# Round 6: the one-sided (ipc) KV transport on one GPU -- in-process loopback
# (kv_copy_blocks into the decode engine's tensor) and two bench processes
# (the prefill rank writes through the decode rank's IPC mapping).
set -o pipefail
out=${1:-gpurun_out/r6_ipc}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_disagg_loopback.py -m gpu -k "one_sided or ipc or device_path" > "$out/tests.log" 2>&1
rc=$?
tail -15 "$out/tests.log"
exit $rc
