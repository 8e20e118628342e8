set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "prefill" > gpurun_out/t_kern.log 2>&1 || { echo KERNEL_TEST_FAIL; tail -40 gpurun_out/t_kern.log; exit 1; }
tail -1 gpurun_out/t_kern.log
for i in 1 2; do timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/mb_attn.json 2> gpurun_out/mb_attn.err && python -c "import json;d=json.load(open('gpurun_out/mb_attn.json'));print({k:v.get('TFLOPs',v.get('TB/s')) for k,v in d.items()})"; done
