#!/bin/bash
# Disagg vs agg projection for Llama-3-70B (the reference's comparison model, docs/architecture.md:57-61) from
# single-MI355X TP1 roles on the final round-5 kernels (MFMA decode attention at GQA group 8):
#   a: prefill role (prompts/s), aggregated sweep, decode role with every prompt remote (q = 1)
#   b: decode role with 75 % / 50 % of the prompts remote
# Concurrency capped at 96: 70B bf16 weights (141 GB) + 96 x 3214-token KV (99 GB) fit 0.9 x 288 GB.
set -o pipefail
mkdir -p gpurun_out/proj70
O=gpurun_out/proj70
SW="--model llama3-70b --steps 6 --warmup 2"
if [ "$1" = a ]; then
  timeout -k 10 300 python tools/role_bench.py --role prefill --model llama3-70b --budget 16384 --steps 10 --warmup 3 \
    > $O/prefill_role.json 2> $O/prefill_role.err || { tail -20 $O/prefill_role.err; exit 1; }
  cat $O/prefill_role.json
  timeout -k 10 700 python bench.py --sweep 8,16,32,64,96 $SW > $O/agg.json 2> $O/agg.err \
    || { tail -20 $O/agg.err; exit 1; }
else
  for q in ${2:-1.0 0.75 0.5}; do
    timeout -k 10 500 python bench.py --sweep 16,32,64,96 --remote-frac $q $SW > $O/q$q.json 2> $O/q$q.err \
      || { tail -20 $O/q$q.err; exit 1; }
  done
fi
