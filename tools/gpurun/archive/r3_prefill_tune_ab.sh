#!/bin/bash
# prefill GEMM bucket tuner: test, then the driver-shaped bench with / without it, interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gemm.py -m gpu -x -q -k "prefill_gemms or model_tune" --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
for i in 1 2; do
  for t in 1 0; do
    DX_PREFILL_TUNE=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 --gemm-report gpurun_out/gemm_pt${t}_$i.json > gpurun_out/ab_pt${t}_$i.json 2> gpurun_out/ab_pt${t}_$i.err || { echo "BENCH FAILED pt=$t"; tail -20 gpurun_out/ab_pt${t}_$i.err; exit 1; }
    echo "prefill_tune=$t run $i: $(python -c "import json;d=json.load(open('gpurun_out/ab_pt${t}_$i.json'));print(d['value'], 'ttft', d['ttft_p50_ms'], 'step_itl', d['step_itl_p50_ms'], 'qps', d['qps'], d['ttft_p50_ms_at_qps'])")"
  done
done
python -c "import json;d=json.load(open('gpurun_out/gemm_pt1_1.json'));print('adopted', [(r['bucket'], r['N'], r['K'], r['lib_us'], r['gemm256_us']) for r in d['prefill'] if r['adopted']])"
