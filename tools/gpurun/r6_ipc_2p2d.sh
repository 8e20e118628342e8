#!/bin/bash
# Round 6: the headline model's disagg bench path over the one-sided transport, 2P2D with all four ranks on the
# one GPU (full Llama-3-8B, shareable decode caches of 16 GB each): preflight + verify + a short window.
# tok/s is NOT a disagg number (four ranks share one device).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6_ipc_2p2d}
mkdir -p $O
DX_PREFILL_TUNE=0 DX_SKINNY=0 GPU_MAX_HW_QUEUES=2 timeout -k 10 900 python -u bench.py --gpus 4 --p2p-backend ipc \
  --model llama3-8b --num-gpu-blocks 2000 --concurrency 16 --steps 3 --warmup 1 --iters-per-step 10 \
  --qps-segment 0 --verify-tokens 2 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
grep -E "preflight|verify" $O/bench.err | tail -4
