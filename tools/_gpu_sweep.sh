set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/t_engine.log 2>&1 || { echo ENGINE_TEST_FAIL; tail -30 gpurun_out/t_engine.log; exit 1; }
tail -3 gpurun_out/t_engine.log
for cfg in "--policy chunked --max-batched-tokens 8192 --concurrency 128" "--policy chunked --max-batched-tokens 16384 --concurrency 128" "--policy chunked --max-batched-tokens 8192 --concurrency 192" "--policy chunked --max-batched-tokens 8192 --concurrency 256" "--policy prefill-first --concurrency 128"; do
  timeout -k 10 400 python bench.py --steps 300 --warmup 150 $cfg > gpurun_out/b.json 2> gpurun_out/b.err || { echo BENCH_FAIL $cfg; tail -20 gpurun_out/b.err; exit 1; }
  echo "$cfg :: $(cat gpurun_out/b.json)" >> gpurun_out/sweep.txt
done
cat gpurun_out/sweep.txt
