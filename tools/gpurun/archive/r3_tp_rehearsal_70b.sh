#!/bin/bash
# 1P(tp2)+1D(tp2) disaggregated bench of the Llama-3-70B architecture truncated to 20 of its 80
# layers (real 70B layer shapes: 64 q / 8 kv heads split over TP2, hidden 8192, MLP 28672), all 4
# ranks on ONE GPU (host-staged KV over gloo, custom xGMI all-reduce/all-gather inside the TP
# groups) + --verify-tokens against a TP1 aggregated engine.  A rehearsal of the TP data plane at
# 70B shapes, not a 70B throughput number.
set -o pipefail
mkdir -p gpurun_out
export DX_BENCH_VERBOSE=1
timeout -k 10 1000 python bench.py --model llama3-70b@20 --gpus 4 --tp 2 --p2p-backend gloo --steps 4 --warmup 1 \
  --concurrency 8 --num-gpu-blocks 2000 --max-batched-tokens 8192 --verify-tokens 2 --qps-seconds 6 \
  > gpurun_out/r3_tp2_70b_rehearsal.json 2> gpurun_out/r3_tp2_70b_rehearsal.err || { echo "REHEARSAL FAILED"; tail -40 gpurun_out/r3_tp2_70b_rehearsal.err; exit 1; }
tail -1 gpurun_out/r3_tp2_70b_rehearsal.json
