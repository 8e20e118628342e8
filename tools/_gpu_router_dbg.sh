set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
DX_SLOW_REQUEST_S=0.8 timeout -k 20 600 python -u tools/router_bench.py --modes random --workers 2 --num-gpu-blocks 384 --groups 16 --prefix-len 2048 --isl 2304 --osl 16 --concurrency 16 --requests-per-conc 10 --out gpurun_out/router_dbg_$i.json > gpurun_out/router_dbg_$i.log 2>&1 || { echo ROUTER_FAIL; tail -30 gpurun_out/router_dbg_$i.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/router_dbg_$i.json'));print({m:{k:v[k] for k in ('wall_s','ttft_mean_ms','ttft_p50_ms','ttft_max_ms','ttft_over_1s')} for m,v in d['modes'].items()})"
grep -c "slow request" gpurun_out/router_dbg_$i.log || true
done
