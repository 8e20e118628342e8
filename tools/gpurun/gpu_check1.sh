set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err && cat gpurun_out/bench_n1.json &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 100 --warmup 20 --p2p-backend gloo --concurrency 32 --num-gpu-blocks 4000 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err && cat gpurun_out/bench_n2.json
