#!/bin/bash
# Disagg vs agg projection for Llama-3-70B at the reference's precision (FP8: w8a8 e4m3fn projections + e4m3fn
# KV cache; docs/architecture.md:57-61 compares 70B FP8) from single-MI355X TP1 roles:
#   a: prefill role (prompts/s) + aggregated sweep;  b: decode role with 100 % / 75 % of the prompts remote;
#   c: decode role with 50 % remote.
# 70 GB of fp8 weights leave ~190 GB of KV (160 KiB per token): concurrency up to 192.
set -o pipefail
mkdir -p gpurun_out/proj70f
O=gpurun_out/proj70f
Q="--quantization fp8 --kv-cache-dtype fp8"
SW="--model llama3-70b --steps 6 --warmup 2 $Q"
if [ "$1" = a ]; then
  timeout -k 10 300 python tools/role_bench.py --role prefill --model llama3-70b --budget 16384 --steps 10 --warmup 3 $Q \
    > $O/prefill_role.json 2> $O/prefill_role.err || { tail -20 $O/prefill_role.err; exit 1; }
  cat $O/prefill_role.json
  timeout -k 10 870 python bench.py --sweep 8,16,32,64,128 $SW > $O/agg.json 2> $O/agg.err \
    || { tail -20 $O/agg.err; exit 1; }
  tail -c 600 $O/agg.json
elif [ "$1" = b ]; then
  for q in 1.0 0.75; do
    timeout -k 10 500 python bench.py --sweep 16,32,64,128 --remote-frac $q $SW > $O/q$q.json 2> $O/q$q.err \
      || { tail -20 $O/q$q.err; exit 1; }
  done
else
  timeout -k 10 500 python bench.py --sweep 16,32,64,128 --remote-frac 0.5 $SW > $O/q0.5.json 2> $O/q0.5.err \
    || { tail -20 $O/q0.5.err; exit 1; }
fi
