set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# 1P1D sharing the one GPU: KV host-staged over gloo (functional rehearsal of the layer-streamed path)
timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 2 --p2p-backend gloo --concurrency 64 --num-gpu-blocks 4000 --gpu-mem-util 0.4 > gpurun_out/r2_bench_n2.json 2> gpurun_out/r2_bench_n2.err
rc=$?; echo "bench n2 rc=$rc"; tail -1 gpurun_out/r2_bench_n2.json; grep -v "^\[bench\] step" gpurun_out/r2_bench_n2.err | tail -5; exit $rc
