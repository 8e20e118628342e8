#!/bin/bash
# the benchmarked scheduler policy is the served one.  On one MI355X: (a) the driver's bench
# command, (b) `run in=http out=native` with its DEFAULT scheduler policy (engine/policy.py SERVING_DEFAULTS, the
# same the bench uses) under tools/loadgen.py at C=128 streaming chat (raw client on the same box); the loadgen's
# steady-state window (all 128 streams in flight) is compared with the bench's tok/s.
set -o pipefail
mkdir -p gpurun_out
ROOT=$PWD
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_hvb_bench.json 2> gpurun_out/r5_hvb_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r5_hvb_bench.err; exit 1; }
tail -1 gpurun_out/r5_hvb_bench.json | cut -c1-200
ready() {  # $1 url, $2 pid
  for i in $(seq 1 240); do
    curl -s -m 2 "$1/v1/models" | grep -q llama3-8b && return 0
    kill -0 "$2" 2>/dev/null || return 1
    sleep 1
  done
  return 1
}
DYN_LOG=warning timeout -k 10 600 python -m dynamo_exp_amd.cli.run in=http out=native --model-path llama3-8b \
  --model-name llama3-8b --http-port 8123 --max-num-seqs 128 > gpurun_out/r5_hvb_server.log 2>&1 &
SRV=$!
ready http://127.0.0.1:8123 $SRV || { echo "server not ready"; tail -20 gpurun_out/r5_hvb_server.log; kill $SRV; exit 1; }
# --isl 2909: the Llama-3.1 chat template (default system header) adds 91 tokens, so the engine sees 3000-token
# prompts as in the bench (measured through the preprocessor)
timeout -k 10 420 python tools/loadgen.py --url http://127.0.0.1:8123 --model llama3-8b --isl 2909 --osl 150 \
  --isl-unit chars --concurrency 128 --requests-per-conc 8 --warmup-per-conc 2 --client raw \
  --out gpurun_out/r5_hvb_http_c128.json > gpurun_out/r5_hvb_http_c128.log 2>&1; RC=$?
kill $SRV; wait $SRV 2>/dev/null
tail -1 gpurun_out/r5_hvb_http_c128.log
exit $RC
