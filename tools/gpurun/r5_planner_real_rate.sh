#!/bin/bash
# GPU suite on the current tree, then the planner's predictive "rate" policy scaling REAL HIP engines on one
# MI355X (tools/planner_gpu_check.py --policy rate): 1P1D Llama-3-8B sharing the GPU, overload -> add
# PrefillWorker(s) -> the new engines serve -> quiet -> remove.
set -o pipefail
mkdir -p gpurun_out/r5plr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5plr/suite.log 2>&1 || { echo "SUITE FAILED"; tail -30 gpurun_out/r5plr/suite.log; exit 1; }
tail -2 gpurun_out/r5plr/suite.log
timeout -k 10 1000 python tools/planner_gpu_check.py --policy rate --out gpurun_out/r5plr/planner_real_engines_rate.json \
  > gpurun_out/r5plr/log.txt 2>&1; rc=$?
tail -5 gpurun_out/r5plr/log.txt
exit $rc
