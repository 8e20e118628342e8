#!/bin/bash
# Round 6: KV-aware vs random routing, the reference's ISL 4K / OSL 800 shape under an open-loop Poisson load
# (6 req/s for 120 s per mode) where prefix hits decide how much of the GPU prefill takes: 2 Llama-3-8B workers
# sharing one MI355X, 128 shared-prefix groups of 3584 tokens (each worker's KV pool holds about half of them
# beside its active requests), 512 unique tokens per prompt.
set -o pipefail
O=${1:-gpurun_out/r6_router_open}
mkdir -p $O
timeout -k 10 1100 python -u tools/router_bench.py --workers 2 --isl 4096 --prefix-len 3584 --osl 800 \
  --max-model-len 5120 --num-gpu-blocks 4800 --max-num-seqs 96 --groups 128 --rate 6 --duration 120 \
  --out $O/router.json > $O/router.log 2>&1 || { echo "ROUTER BENCH FAILED"; tail -40 $O/router.log; exit 1; }
tail -2 $O/router.log
