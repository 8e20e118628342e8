#!/bin/bash
# `run in=http out=native` at C=128 (tools/loadgen.py, raw client, steady-state window) with the engine's
# periodic device-busy log (DX_ENGINE_STATS_S), A/B over the engine thread's GIL switch interval.
set -o pipefail
mkdir -p gpurun_out/http_ab
O=gpurun_out/http_ab
ready() {  # $1 url, $2 pid
  for i in $(seq 1 240); do
    curl -s -m 2 "$1/v1/models" | grep -q llama3-8b && return 0
    kill -0 "$2" 2>/dev/null || return 1
    sleep 1
  done
  return 1
}
for sw in ${@:-0.0005 0.0001}; do
  DX_ENGINE_STATS_S=5 DX_GIL_SWITCH_INTERVAL_S=$sw DYN_LOG=info timeout -k 10 400 python -m dynamo_exp_amd.cli.run \
    in=http out=native --model-path llama3-8b --model-name llama3-8b --http-port 8123 --max-num-seqs 128 \
    > $O/server_sw$sw.log 2>&1 &
  SRV=$!
  ready http://127.0.0.1:8123 $SRV || { echo "server not ready"; tail -20 $O/server_sw$sw.log; kill $SRV; exit 1; }
  timeout -k 10 300 python tools/loadgen.py --url http://127.0.0.1:8123 --model llama3-8b --isl 3000 --osl 150 \
    --isl-unit chars --concurrency 128 --requests-per-conc 6 --warmup-per-conc 2 --client raw \
    --out $O/http_sw$sw.json > $O/http_sw$sw.log 2>&1; RC=$?
  kill $SRV; wait $SRV 2>/dev/null
  tail -1 $O/http_sw$sw.log | cut -c1-400
  grep "engine stats" $O/server_sw$sw.log | tail -4
  [ $RC -eq 0 ] || exit $RC
done
