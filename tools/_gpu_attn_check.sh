set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/t_kern.log 2>&1 || { echo KERNEL_TEST_FAIL; tail -40 gpurun_out/t_kern.log; exit 1; }
tail -2 gpurun_out/t_kern.log
timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/mb_attn.json 2> gpurun_out/mb_attn.err || { echo MB_FAIL; tail gpurun_out/mb_attn.err; exit 1; }
timeout -k 10 300 python tools/microbench.py --what decode > gpurun_out/mb_dec.json 2> gpurun_out/mb_dec.err || { echo MB_FAIL; tail gpurun_out/mb_dec.err; exit 1; }
cat gpurun_out/mb_attn.json gpurun_out/mb_dec.json
