set -o pipefail
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=2
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 200 --warmup 50 --p2p-backend gloo --concurrency 64 --num-gpu-blocks 4500 > gpurun_out/bench_n2_shared.json 2> gpurun_out/bench_n2_shared.err && cat gpurun_out/bench_n2_shared.json || { tail -30 gpurun_out/bench_n2_shared.err; exit 1; }
grep "per-rank" gpurun_out/bench_n2_shared.err | tail -1
