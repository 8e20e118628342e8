#!/bin/bash
# Round 6: the N = 8 disagg layout (4P4D, TP1) over the one-sided transport with all eight ranks on the one GPU
# (Llama-3-8B at 8 layers): 16 pair preflights, token verification, a short window.  Functional, not a number.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6_ipc_4p4d}
mkdir -p $O
DX_PREFILL_TUNE=0 DX_SKINNY=0 GPU_MAX_HW_QUEUES=2 timeout -k 10 900 python -u bench.py --gpus 8 --p2p-backend ipc \
  --model llama3-8b@8 --num-gpu-blocks 800 --concurrency 8 --steps 2 --warmup 1 --iters-per-step 10 \
  --qps-segment 0 --verify-tokens 2 --no-graph > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
grep '^{' $O/bench.json | tail -1 | cut -c1-400
grep -E "preflight ok|verify" $O/bench.err | tail -2 | cut -c1-300
