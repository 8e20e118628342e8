#!/bin/bash
# Round 6: a two-sided KV path failing its preflight falls back to the one-sided transport.
set -o pipefail
out=${1:-gpurun_out/r6_fallback}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_disagg_loopback.py -m gpu -k "falls_back" > "$out/tests.log" 2>&1
rc=$?
tail -12 "$out/tests.log"
exit $rc
