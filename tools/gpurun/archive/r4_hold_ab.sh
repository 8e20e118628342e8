#!/bin/bash
# step-composition A/B on one GPU (bench.py driver command): default vs --prefill-whole-prompts 1; AB="run ..." overrides
set -o pipefail
OUT=${1:-gpurun_out/hold_ab}
mkdir -p "$OUT"
run() {  # name, extra flags
  echo "[ab] $1 $(date +%T)"
  timeout -k 10 420 python bench.py "${@:2}" > "$OUT/$1.json" 2> "$OUT/$1.err" || return 1
  python -c "import json,sys;d=json.load(open('$OUT/$1.json'));c=d['config'];print('$1', d['value'], d['ttft_p50_ms'], d.get('ttft_p50_ms_at_qps'), d.get('ttft_p99_ms_at_qps'), c['mixed_iters'], c['decode_iters'], c.get('prefill_step_tokens_mean'))"
}
if [ -n "$AB" ]; then eval "$AB"; else
run base && run whole --prefill-whole-prompts 1 && run base2 && run whole2 --prefill-whole-prompts 1
fi
