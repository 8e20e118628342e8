set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ov
run() {  # name, env
  env $2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ov/$1.json 2> gpurun_out/ov/$1.err
  rc=$?; echo "$1 rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/ov/$1.json').read().strip().splitlines()[-1]); print(d['value'], d['ttft_p50_ms'], d.get('step_itl_p50_ms'))" 2>/dev/null)"; return $rc
}
run off DX_OVERLAP_DECODE_ATTN=0 && run on DX_OVERLAP_DECODE_ATTN=1 && run off2 DX_OVERLAP_DECODE_ATTN=0 && run on2 DX_OVERLAP_DECODE_ATTN=1
