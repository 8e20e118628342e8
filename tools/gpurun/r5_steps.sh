#!/bin/bash
# Round 5: rocprofv3 kernel trace (csv) of the headline bench's closed-loop window -> per-step breakdown and the
# top-kernel summary (after the MFMA decode attention and the in-wave decode merge).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r5s}
mkdir -p $OUT/steps
timeout -k 10 500 rocprofv3 --kernel-trace -d $OUT/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 > $OUT/steps/bench.json 2> $OUT/steps/bench.err
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find $OUT/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > $OUT/steps/breakdown.txt 2>&1
python3 tools/prof_summary.py "$k" 30 > $OUT/steps/summary.txt 2>&1
rm -f "$k"
cat $OUT/steps/breakdown.txt
