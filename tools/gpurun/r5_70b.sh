#!/bin/bash
# config 4's model on the current tree, one MI355X.
#  (a) one Llama-3-70B TP4 rank's projection shapes through the engine's decode-GEMM tuner + prefill GEMM rates;
#  (b) prefill / decode attention at the TP4 rank's 16 q / 2 KV heads;
#  (c) Llama-3-70B TP1 bench at C = 64 (round 1: 362 tok/s bf16);
#  (d) Llama-3-70B@20 layers 1P(tp2)1D(tp2) rehearsal, four ranks on the one GPU (host-staged KV, gloo TP).
set -o pipefail
mkdir -p gpurun_out/r5_70b
O=gpurun_out/r5_70b
timeout -k 10 420 python tools/tp_shapes_bench.py --model llama3-70b --tp 4 --out $O/tp4_shapes.json \
  > $O/tp4_shapes.log 2>&1 || { tail -20 $O/tp4_shapes.log; exit 1; }
tail -2 $O/tp4_shapes.log
timeout -k 10 300 python tools/microbench.py --what attn --heads 16,2 > $O/attn_16_2.json 2> $O/attn_16_2.err \
  || { tail -20 $O/attn_16_2.err; exit 1; }
timeout -k 10 600 python bench.py --model llama3-70b --concurrency 64 --steps 10 --warmup 3 \
  > $O/bench_70b_tp1.json 2> $O/bench_70b_tp1.err || { tail -20 $O/bench_70b_tp1.err; exit 1; }
tail -1 $O/bench_70b_tp1.json | cut -c1-300
