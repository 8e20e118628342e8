#!/bin/bash
# Round 4: rocprofv3 kernel trace of the one-GPU loopback 1P1D run -> per-forward GPU busy / idle gaps
# (phase A: prefill forwards without transfer; phase B: the same with the KV streamed per layer group).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4e}/lb
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT -o lb --output-format csv -- python3 tools/loopback_disagg.py --prompts 24 --out $OUT/loopback.json > $OUT/loopback.log 2>&1
rc=$?; echo "rocprof loopback rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/gap_report.py "$k" 32 > $OUT/gaps.txt 2>&1
rm -f "$k"
