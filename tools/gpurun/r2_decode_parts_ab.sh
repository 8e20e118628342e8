set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dp
run() {  # name, env
  env $2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dp/$1.json 2> gpurun_out/dp/$1.err
  rc=$?; echo "$1 rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/dp/$1.json').read().strip().splitlines()[-1]); print(d['value'], d['ttft_p50_ms'], d.get('step_itl_p50_ms'))" 2>/dev/null)"; return $rc
}
run w2048 DX_DECODE_WGS=2048 && run w1024 DX_DECODE_WGS=1024 && run w3072 DX_DECODE_WGS=3072 && run w2048b DX_DECODE_WGS=2048 && run w1024b DX_DECODE_WGS=1024
