#!/bin/bash
# Round 6: the deep-stream SwiGLU form's numerics, the driver's bench command with the decode-GEMM tuning table, and
# KV-aware vs random routing under a prefill-contended load with the reference's ISL 4K / OSL 800 shape.
set -o pipefail
O=${1:-gpurun_out/r6b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_skinny_gemm.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/skinny_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/skinny_tests.log; exit 1; }
tail -3 $O/skinny_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --gemm-report $O/gemm_report.json > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 1000 python -u tools/router_bench.py --workers 2 --isl 4096 --prefix-len 3584 --osl 800 \
  --max-model-len 5120 --num-gpu-blocks 4200 --groups 40 --concurrency 96 --requests-per-conc 2 \
  --warmup-per-conc 1 --out $O/router.json > $O/router.log 2>&1 || { echo "ROUTER BENCH FAILED"; tail -40 $O/router.log; exit 1; }
tail -2 $O/router.log
