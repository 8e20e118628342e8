set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kv_fp8.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/kv_fp8_tests2.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/kv_fp8_tests2.log; exit 1; }
tail -1 gpurun_out/kv_fp8_tests2.log
timeout -k 10 200 python -u -m tools.kv_fp8_probe 2>&1 | grep -v amdgpu.ids || exit 1
for kv in fp8 auto; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --kv-cache-dtype $kv > gpurun_out/bench_kv_$kv.json 2> gpurun_out/bench_kv_$kv.err || { echo "BENCH FAILED $kv"; tail -20 gpurun_out/bench_kv_$kv.err; exit 1; }
  echo "kv=$kv: $(python -c "import json;d=json.load(open('gpurun_out/bench_kv_$kv.json'));print(d['value'], d['dtype'], 'ttft', d['ttft_p50_ms'], 'step_itl', d['step_itl_p50_ms'], 'qps', d['qps'], d['ttft_p50_ms_at_qps'])")"
done
