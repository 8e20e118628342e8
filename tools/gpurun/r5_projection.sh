#!/bin/bash
# measurements for tools/disagg_projection.py on one MI355X at the current kernels --
# the prefill role (prompts/s), the aggregated concurrency sweep and decode-role sweeps with a fraction q of the
# prompts remotely prefilled (q = 1: always remote; q < 1: conditional disaggregation's decode GPU).
set -o pipefail
mkdir -p gpurun_out/proj
O=gpurun_out/proj
timeout -k 10 240 python tools/role_bench.py --role prefill --budget 16384 --steps 40 --warmup 8 \
  > $O/prefill_role.json 2> $O/prefill_role.err || { tail -20 $O/prefill_role.err; exit 1; }
cat $O/prefill_role.json
SW="--steps 10 --warmup 3"
timeout -k 10 600 python bench.py --sweep 8,16,32,64,96,128,192,256 $SW > $O/agg.json 2> $O/agg.err \
  || { tail -20 $O/agg.err; exit 1; }
for q in 1.0 0.75 0.5; do
  timeout -k 10 600 python bench.py --sweep 32,64,128,192,256,384 --remote-frac $q $SW > $O/q$q.json 2> $O/q$q.err \
    || { tail -20 $O/q$q.err; exit 1; }
done
P=$(python -c "import json; print(json.load(open('$O/prefill_role.json'))['prompts_s'])")
python tools/disagg_projection.py --agg $O/agg.json --decode $O/q1.0.json $O/q0.75.json $O/q0.5.json \
  --prefill-prompts-s $P --out $O/projection.json
