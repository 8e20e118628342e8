#!/bin/bash
# headline bench A/B: decode GEMM tuner with / without the register-streamed kernel, interleaved
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    DX_VSTREAM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --gemm-report gpurun_out/gemm_vs${v}_$i.json > gpurun_out/ab_vs${v}_$i.json 2> gpurun_out/ab_vs${v}_$i.err || { echo "BENCH FAILED vs=$v"; tail -20 gpurun_out/ab_vs${v}_$i.err; exit 1; }
    echo "vs=$v run $i: $(python -c "import json;d=json.load(open('gpurun_out/ab_vs${v}_$i.json'));print(d['value'], d['step_itl_p50_ms'], d['ttft_p50_ms'])")"
  done
done
