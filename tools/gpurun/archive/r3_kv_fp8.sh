#!/bin/bash
# fp8 KV cache: numerics (new + the attention/rope/engine suites the signature change touches), then the bench with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kv_fp8.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/kv_fp8_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/kv_fp8_tests.log; exit 1; }
tail -3 gpurun_out/kv_fp8_tests.log
for kv in fp8 auto; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --kv-cache-dtype $kv > gpurun_out/bench_kv_$kv.json 2> gpurun_out/bench_kv_$kv.err || { echo "BENCH FAILED $kv"; tail -20 gpurun_out/bench_kv_$kv.err; exit 1; }
  echo "kv=$kv: $(python -c "import json;d=json.load(open('gpurun_out/bench_kv_$kv.json'));print(d['value'], d['dtype'], 'ttft', d['ttft_p50_ms'], 'step_itl', d['step_itl_p50_ms'], 'qps', d['qps'], d['ttft_p50_ms_at_qps'])")"
done
