#!/bin/bash
# Round 6: KV-aware vs random routing on the current engine with the reference's workload shape (VERDICT r5
# missing #5 / next #9): ISL ~4K with a 3.5K shared prefix per group, OSL 800 (docs/architecture.md:78-87 of the
# reference: ISL 4K / OSL 800), 2 Llama-3-8B workers sharing one MI355X, 16 prefix groups, closed loop C = 16.
set -o pipefail
O=${1:-gpurun_out/r6_router}
mkdir -p $O
timeout -k 10 1000 python -u tools/router_bench.py --workers 2 --isl 4096 --prefix-len 3584 --osl 800 \
  --max-model-len 5120 --num-gpu-blocks 1280 --groups 16 --concurrency 16 --requests-per-conc 4 \
  --warmup-per-conc 1 --out $O/router.json > $O/router.log 2>&1 || { echo "ROUTER BENCH FAILED"; tail -40 $O/router.log; exit 1; }
tail -5 $O/router.log
