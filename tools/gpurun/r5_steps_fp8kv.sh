#!/bin/bash
# rocprofv3 kernel trace of the bench window with the opt-in fp8 KV cache -> per-step breakdown (not the headline)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5s8
mkdir -p $OUT/steps
timeout -k 10 500 rocprofv3 --kernel-trace -d $OUT/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 --kv-cache-dtype fp8 > $OUT/steps/bench.json 2> $OUT/steps/bench.err
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find $OUT/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > $OUT/steps/breakdown.txt 2>&1
rm -f "$k"
cat $OUT/steps/breakdown.txt
