set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
DX_DUMP_AFTER=500 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --p2p-backend gloo --num-gpu-blocks 3000 --steps 60 --warmup 20 --concurrency 16 > gpurun_out/disagg2.json 2> gpurun_out/disagg2.err || { echo DISAGG_FAIL; tail -40 gpurun_out/disagg2.err; exit 1; }
cat gpurun_out/disagg2.json
