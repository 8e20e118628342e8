set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
timeout -k 10 600 python bench.py --model llama3-70b --concurrency 32 --steps 100 --warmup 40 > gpurun_out/b70.json 2> gpurun_out/b70.err || { echo B70_FAIL; tail -20 gpurun_out/b70.err; exit 1; }
cat gpurun_out/b70.json
timeout -k 10 400 python bench.py --model deepseek-r1-distill-llama-8b --steps 100 --warmup 40 > gpurun_out/bds.json 2> gpurun_out/bds.err || { echo BDS_FAIL; tail -20 gpurun_out/bds.err; exit 1; }
cat gpurun_out/bds.json
