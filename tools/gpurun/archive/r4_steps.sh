#!/bin/bash
# Round 4: rocprofv3 kernel traces (csv) of (1) the headline bench's closed-loop window -> per-step breakdown,
# (2) the one-GPU loopback 1P1D run -> GPU busy / idle gaps while prefill forwards stream their KV.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4d}
mkdir -p $OUT/steps $OUT/lb
timeout -k 10 500 rocprofv3 --kernel-trace -d $OUT/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 > $OUT/steps/bench.json 2> $OUT/steps/bench.err
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find $OUT/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > $OUT/steps/breakdown.txt 2>&1
python3 tools/prof_summary.py "$k" 30 > $OUT/steps/summary.txt 2>&1
rm -f "$k"
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/lb -o lb --output-format csv -- python3 tools/loopback_disagg.py --prompts 24 --out $OUT/lb/loopback.json > $OUT/lb/loopback.log 2>&1
rc=$?; echo "rocprof loopback rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find $OUT/lb -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$k" 30 > $OUT/lb/summary.txt 2>&1
python3 tools/gap_report.py "$k" 32 > $OUT/lb/gaps.txt 2>&1
rm -f "$k"
