set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
run() {  # name, extra bench flags
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $2 > gpurun_out/sweep/$1.json 2> gpurun_out/sweep/$1.err
  rc=$?; echo "$1 rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$1.json').read().strip().splitlines()[-1]); print(d['value'], d['ttft_p50_ms'], d.get('step_itl_p50_ms'))" 2>/dev/null)"; return $rc
}
run base "" && run mpt12k "--min-prefill-tokens 12000 --max-prefill-delay 0.4" && \
run mbt12k "--max-batched-tokens 12288 --min-prefill-tokens 12000 --max-prefill-delay 0.4" && \
run mpt6k "--min-prefill-tokens 6000 --max-prefill-delay 0.25" && run mbt16k "--max-batched-tokens 16384 --min-prefill-tokens 16000 --max-prefill-delay 0.5"
