#!/bin/bash
# rocprofv3 kernel trace of the headline bench (closed-loop window only) -> per-step breakdown + kernel table.
set -o pipefail
mkdir -p gpurun_out/steps
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 > gpurun_out/steps/bench.json 2> gpurun_out/steps/bench.err
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/steps/bench.json; [ $rc -eq 0 ] || exit $rc
k=$(find gpurun_out/steps -name "*kernel_trace.csv" | head -1); echo "trace: $k"
python3 tools/step_breakdown.py "$k" 10 > gpurun_out/steps/breakdown.txt 2>&1; cat gpurun_out/steps/breakdown.txt
python3 tools/prof_summary.py "$k" 30 > gpurun_out/steps/summary.txt 2>&1
rm -f "$k"
