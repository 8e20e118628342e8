#!/bin/bash
# Driver-shaped bench with the opt-in fp8 (e4m3fn) KV cache next to its bf16-cache twin on the same box
# (not the headline: the headline is bf16 everywhere).
set -o pipefail
mkdir -p gpurun_out/r5kv8
O=gpurun_out/r5kv8
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --kv-cache-dtype fp8 > $O/fp8.json 2> $O/fp8.err \
  || { tail -20 $O/fp8.err; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bf16.json 2> $O/bf16.err || { tail -20 $O/bf16.err; exit 1; }
for f in fp8 bf16; do tail -1 $O/$f.json | cut -c1-260; echo; done
