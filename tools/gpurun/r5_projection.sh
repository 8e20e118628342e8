#!/bin/bash
# measurements for tools/disagg_projection.py on one MI355X at the current kernels --
# part a: the prefill role (prompts/s), the aggregated concurrency sweep, the pure decode role (q = 1);
# part b: decode-role sweeps with a fraction q of the prompts remotely prefilled (conditional disaggregation's
# decode GPU).  The projection itself runs on the CPU afterwards (gpurun_out/ does not travel to the box):
#   python tools/disagg_projection.py --agg gpurun_out/proj/agg.json --decode gpurun_out/proj/q*.json \
#     --prefill-prompts-s <prefill_role.json prompts_s> --out profiles/r5_disagg_projection.json
set -o pipefail
mkdir -p gpurun_out/proj
O=gpurun_out/proj
SW="--steps 10 --warmup 3"
if [ "$1" = a ]; then
  timeout -k 10 240 python tools/role_bench.py --role prefill --budget 16384 --steps 40 --warmup 8 \
    > $O/prefill_role.json 2> $O/prefill_role.err || { tail -20 $O/prefill_role.err; exit 1; }
  cat $O/prefill_role.json
  timeout -k 10 500 python bench.py --sweep 8,16,32,64,96,128,192,256 $SW > $O/agg.json 2> $O/agg.err \
    || { tail -20 $O/agg.err; exit 1; }
  timeout -k 10 400 python bench.py --sweep 32,64,128,192,256,384 --remote-frac 1.0 $SW > $O/q1.0.json \
    2> $O/q1.0.err || { tail -20 $O/q1.0.err; exit 1; }
else
  for q in 0.75 0.5; do
    timeout -k 10 500 python bench.py --sweep 64,128,192,256,384 --remote-frac $q $SW > $O/q$q.json 2> $O/q$q.err \
      || { tail -20 $O/q$q.err; exit 1; }
  done
fi
