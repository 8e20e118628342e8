#!/bin/bash
# Token budget A/B on the final round-5 kernels (driver-shaped runs, one box): 8192 (serving default) vs 12288 vs
# 16384 tokens per step, the prefill-batching threshold scaled with the budget.
set -o pipefail
mkdir -p gpurun_out/r5bud
O=gpurun_out/r5bud
for cfg in "8192 8000" "12288 12000" "16384 16000"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --max-batched-tokens $1 --min-prefill-tokens $2 \
    > $O/b$1.json 2> $O/b$1.err || { tail -20 $O/b$1.err; exit 1; }
  tail -1 $O/b$1.json | cut -c1-200; echo
done
