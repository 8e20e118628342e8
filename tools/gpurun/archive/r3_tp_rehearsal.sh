#!/bin/bash
# 1P(tp2)+1D(tp2) disaggregated bench with all 4 ranks on ONE GPU (host-staged KV over gloo,
# custom xGMI all-reduce/all-gather inside the TP groups): the TP data plane end to end on a
# real MI355X, plus --verify-tokens (fixed prompts through remote prefill == TP1 aggregated).
set -o pipefail
mkdir -p gpurun_out
export DX_BENCH_VERBOSE=1
timeout -k 10 1000 python bench.py --gpus 4 --tp 2 --p2p-backend gloo --steps 6 --warmup 2 --concurrency 16 \
  --num-gpu-blocks 3000 --max-batched-tokens 8192 --verify-tokens 2 --qps-seconds 6 \
  > gpurun_out/r3_tp2_rehearsal.json 2> gpurun_out/r3_tp2_rehearsal.err || { echo "REHEARSAL FAILED"; tail -40 gpurun_out/r3_tp2_rehearsal.err; exit 1; }
cat gpurun_out/r3_tp2_rehearsal.json
