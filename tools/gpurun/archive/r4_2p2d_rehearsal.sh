#!/bin/bash
# 2P2D disaggregated bench with all 4 ranks on ONE GPU (host-staged KV over gloo): the xPyD layout the
# driver's N=4 run uses, with its pre-flight (one WRITE + one READ per (prefill, decode) pair, 4 pairs)
# and --verify-tokens, after the round-4 changes.
set -o pipefail
mkdir -p gpurun_out
export DX_BENCH_VERBOSE=1
timeout -k 10 900 python bench.py --gpus 4 --p2p-backend gloo --steps 4 --warmup 2 --concurrency 8 \
  --num-gpu-blocks 3000 --verify-tokens 2 --qps-seconds 6 \
  > gpurun_out/r4_2p2d_rehearsal.json 2> gpurun_out/r4_2p2d_rehearsal.err || { echo "REHEARSAL FAILED"; tail -40 gpurun_out/r4_2p2d_rehearsal.err; exit 1; }
cat gpurun_out/r4_2p2d_rehearsal.json
grep -E "preflight|verify" gpurun_out/r4_2p2d_rehearsal.err | tail -12
