set -o pipefail
mkdir -p gpurun_out
timeout -k 20 900 python -u tools/router_bench.py --workers 4 --num-gpu-blocks 384 --groups 32 --prefix-len 2048 --isl 2304 --osl 32 --concurrency 32 --requests-per-conc 10 --out gpurun_out/router_bench4.json > gpurun_out/router_bench4.log 2>&1; RC=$?
tail -1 gpurun_out/router_bench4.log
exit $RC
