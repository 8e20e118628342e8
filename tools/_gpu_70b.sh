set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --model llama3-70b --concurrency 64 --steps 200 --warmup 50 > gpurun_out/b70_bf16.json 2> gpurun_out/b70_bf16.err || { echo B70_FAIL; tail -20 gpurun_out/b70_bf16.err; exit 1; }
cat gpurun_out/b70_bf16.json
timeout -k 10 900 python -u bench.py --model llama3-70b --quantization fp8 --concurrency 64 --steps 200 --warmup 50 > gpurun_out/b70_fp8.json 2> gpurun_out/b70_fp8.err || { echo B70F_FAIL; tail -20 gpurun_out/b70_fp8.err; exit 1; }
cat gpurun_out/b70_fp8.json
