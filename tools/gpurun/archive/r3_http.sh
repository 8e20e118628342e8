#!/bin/bash
# The OpenAI serving path on one MI355X at the bench's load (Llama-3-8B, ISL 3000 / OSL 150, C=128 streaming
# chat, tools/loadgen.py on the same box): (a) single-process `run in=http out=native`, (b) the distributed
# aggregated graph `dynamo serve graphs.agg:Frontend` (frontend -> processor -> worker over the request plane).
set -o pipefail
mkdir -p gpurun_out
ROOT=$PWD
ready() {  # $1 url, $2 pid
  for i in $(seq 1 240); do
    curl -s -m 2 "$1/v1/models" | grep -q llama3-8b && return 0
    kill -0 "$2" 2>/dev/null || return 1
    sleep 1
  done
  return 1
}
DYN_LOG=warning timeout -k 10 600 python -m dynamo_exp_amd.cli.run in=http out=native --model-path llama3-8b \
  --model-name llama3-8b --http-port 8123 --max-num-seqs 128 \
  --extra-engine-args '{"min_prefill_tokens": 8000, "max_prefill_delay": 0.3, "max_num_batched_tokens": 8192}' \
  > gpurun_out/r3_http_server.log 2>&1 &
SRV=$!
ready http://127.0.0.1:8123 $SRV || { echo "server not ready"; tail -20 gpurun_out/r3_http_server.log; kill $SRV; exit 1; }
timeout -k 10 400 python tools/loadgen.py --url http://127.0.0.1:8123 --model llama3-8b --isl 3000 --osl 150 \
  --isl-unit chars --concurrency 128 --requests-per-conc 6 --warmup-per-conc 1 --out gpurun_out/r3_http_c128.json \
  > gpurun_out/r3_http_c128.log 2>&1; RC=$?
kill $SRV; wait $SRV 2>/dev/null
tail -2 gpurun_out/r3_http_c128.log
[ $RC -eq 0 ] || { echo "loadgen (a) failed"; exit $RC; }
cd examples/llm
PYTHONPATH=$ROOT DYN_LOG=warning DYN_STATE_DIR=$ROOT/gpurun_out/serve_state timeout -k 10 600 python -m dynamo_exp_amd.sdk.serve \
  graphs.agg:Frontend -f configs/agg.yaml --Frontend.port=8124 --Worker.max-num-seqs=128 \
  --Worker.max-num-batched-tokens=8192 --Worker.min-prefill-tokens=8000 --Worker.max-prefill-delay=0.3 \
  --control-plane 127.0.0.1:8130 > $ROOT/gpurun_out/r3_serve_agg.log 2>&1 &
SRV=$!
cd $ROOT
ready http://127.0.0.1:8124 $SRV || { echo "graph not ready"; tail -20 gpurun_out/r3_serve_agg.log; kill -- -$SRV 2>/dev/null; kill $SRV; exit 1; }
timeout -k 10 400 python tools/loadgen.py --url http://127.0.0.1:8124 --model llama3-8b --isl 3000 --osl 150 \
  --isl-unit chars --concurrency 128 --requests-per-conc 6 --warmup-per-conc 1 --out gpurun_out/r3_serve_agg_c128.json \
  > gpurun_out/r3_serve_agg_c128.log 2>&1; RC=$?
kill $SRV; wait $SRV 2>/dev/null
tail -2 gpurun_out/r3_serve_agg_c128.log
exit $RC
