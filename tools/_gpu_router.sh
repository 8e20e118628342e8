set -o pipefail
mkdir -p gpurun_out
timeout -k 20 900 python -u tools/router_bench.py --workers 2 --num-gpu-blocks 384 --groups 16 --prefix-len 2048 --isl 2304 --osl 16 --concurrency 16 --requests-per-conc 10 --out gpurun_out/router_bench.json > gpurun_out/router_bench.log 2>&1; RC=$?
tail -5 gpurun_out/router_bench.log
exit $RC
