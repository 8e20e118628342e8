#!/bin/bash
# The planner scaling REAL HIP engines on one MI355X (tools/planner_gpu_check.py): 1P1D Llama-3-8B sharing the GPU,
# overload -> add PrefillWorker -> both prefill engines serve -> quiet -> remove.
set -o pipefail
mkdir -p gpurun_out/r5pl
timeout -k 10 1000 python tools/planner_gpu_check.py --out gpurun_out/r5pl/planner_real_engines.json \
  > gpurun_out/r5pl/log.txt 2>&1; rc=$?
tail -5 gpurun_out/r5pl/log.txt
exit $rc
