#!/bin/bash
# 1P1D disaggregated bench with an fp8 KV cache, both ranks on ONE GPU (host-staged KV over gloo):
# the e4m3 KV bytes through the P->D data plane on a real MI355X, with --verify-tokens
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python bench.py --gpus 2 --p2p-backend gloo --kv-cache-dtype fp8 --steps 6 --warmup 2 \
  --concurrency 32 --num-gpu-blocks 4000 --verify-tokens 2 --qps-seconds 6 \
  > gpurun_out/r3_fp8_1p1d_rehearsal.json 2> gpurun_out/r3_fp8_1p1d_rehearsal.err || { echo "REHEARSAL FAILED"; tail -40 gpurun_out/r3_fp8_1p1d_rehearsal.err; exit 1; }
cat gpurun_out/r3_fp8_1p1d_rehearsal.json
