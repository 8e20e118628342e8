# xPyD rehearsal with every rank on the one GPU (KV host-staged over gloo): 1P1D at C=64/GPU, 2P2D at C=32/GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dis
timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 2 --p2p-backend gloo --concurrency 64 --num-gpu-blocks 4000 --gpu-mem-util 0.4 > gpurun_out/dis/n2.json 2> gpurun_out/dis/n2.err
rc=$?; echo "bench n2 rc=$rc"; tail -1 gpurun_out/dis/n2.json | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 4 --steps 10 --warmup 2 --p2p-backend gloo --concurrency 32 --num-gpu-blocks 3000 --gpu-mem-util 0.2 > gpurun_out/dis/n4.json 2> gpurun_out/dis/n4.err
rc=$?; echo "bench n4 rc=$rc"; tail -1 gpurun_out/dis/n4.json | cut -c1-1500; grep "per-rank" gpurun_out/dis/n4.err | cut -c1-1500; exit $rc
