#!/bin/bash
# Round 6: folded RMSNorm -- kernel numerics + model equivalence, then the driver's bench command with the fold on
# and off (DX_FOLD_NORM=0) on the same box, then a kernel trace of the folded bench window.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6_fold}
mkdir -p $O/steps
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_folded_norm.py \
  tests/test_gemm256.py -m gpu > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_fold.json 2> $O/bench_fold.err || { echo "BENCH FAILED"; tail -20 $O/bench_fold.err; exit 1; }
cat $O/bench_fold.json
DX_FOLD_NORM=0 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_nofold.json 2> $O/bench_nofold.err || { echo "BENCH FAILED"; tail -20 $O/bench_nofold.err; exit 1; }
cat $O/bench_nofold.json
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 > $O/steps/bench.json 2> $O/steps/bench.err || { echo "PROF FAILED"; tail -20 $O/steps/bench.err; exit 1; }
k=$(find $O/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > $O/steps/breakdown.txt 2>&1
python3 tools/prof_summary.py "$k" 30 > $O/steps/summary.txt 2>&1
rm -f "$k"
cat $O/steps/breakdown.txt
