#!/bin/bash
# Round 6: GPU suite + smoke + the driver's bench command + a rocprofv3 kernel trace of the bench window (step
# breakdown and top-kernel summary), one gpurun call; every GPU step has its own limit and ends the script on failure.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6}
mkdir -p $O/steps
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { echo "SUITE FAILED"; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 > $O/steps/bench.json 2> $O/steps/bench.err || { echo "PROF FAILED"; tail -20 $O/steps/bench.err; exit 1; }
k=$(find $O/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > $O/steps/breakdown.txt 2>&1
python3 tools/prof_summary.py "$k" 30 > $O/steps/summary.txt 2>&1
rm -f "$k"
cat $O/steps/breakdown.txt
