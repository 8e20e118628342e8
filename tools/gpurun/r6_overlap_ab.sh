#!/bin/bash
# Round 6: decode attention of a mixed step on the side stream beside the prefill attention (DX_OVERLAP_DECODE_ATTN=1)
# vs serial, same box: driver bench both ways + a kernel trace of the overlapped run.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6_overlap}
mkdir -p $O/steps
DX_OVERLAP_DECODE_ATTN=1 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_overlap.json 2> $O/bench_overlap.err || { echo "BENCH FAILED"; tail -20 $O/bench_overlap.err; exit 1; }
cat $O/bench_overlap.json | cut -c1-200
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_serial.json 2> $O/bench_serial.err || { echo "BENCH FAILED"; tail -20 $O/bench_serial.err; exit 1; }
cat $O/bench_serial.json | cut -c1-200
DX_OVERLAP_DECODE_ATTN=1 timeout -k 10 500 rocprofv3 --kernel-trace -d $O/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 --qps-segment 0 > $O/steps/bench.json 2> $O/steps/bench.err || { echo "PROF FAILED"; tail -20 $O/steps/bench.err; exit 1; }
k=$(find $O/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > $O/steps/breakdown.txt 2>&1
rm -f "$k"
cat $O/steps/breakdown.txt
