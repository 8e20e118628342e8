#!/bin/bash
# Llama-3-70B@20 layers 1P(tp2)1D(tp2) rehearsal, four ranks on the one GPU (host-staged
# KV over gloo; TP collectives over gloo since round 5: ranks sharing a device skip the custom all-reduce).
set -o pipefail
mkdir -p gpurun_out/r5_70b
O=gpurun_out/r5_70b
export DX_BENCH_VERBOSE=1
DX_DUMP_AFTER=840 timeout -k 10 900 python bench.py --gpus 4 --p2p-backend gloo --prefill-tp 2 --decode-tp 2 \
  --model llama3-70b@20 --concurrency 16 --steps 2 --warmup 1 --iters-per-step 10 --num-gpu-blocks 2000 \
  --qps-segment 0 --verify-tokens 2 > $O/rehearsal_70b20_1p1d_tp2.json 2> $O/rehearsal_70b20_1p1d_tp2.err \
  || { tail -30 $O/rehearsal_70b20_1p1d_tp2.err; exit 1; }
tail -1 $O/rehearsal_70b20_1p1d_tp2.json | cut -c1-400
