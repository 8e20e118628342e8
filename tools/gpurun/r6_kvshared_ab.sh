#!/bin/bash
# Round 6: does the VMM-chunked (shareable) KV cache cost anything?  Driver bench with DX_KV_SHARED=1 vs default.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6_kvshared}
mkdir -p $O
DX_KV_SHARED=1 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_shared.json 2> $O/bench_shared.err || { echo "BENCH FAILED"; tail -20 $O/bench_shared.err; exit 1; }
cat $O/bench_shared.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_plain.json 2> $O/bench_plain.err || { echo "BENCH FAILED"; tail -20 $O/bench_plain.err; exit 1; }
cat $O/bench_plain.json
