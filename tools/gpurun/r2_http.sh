set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DYN_LOG=warning timeout -k 10 700 python -m dynamo_exp_amd.cli.run in=http out=native --model-path llama3-8b --model-name llama3-8b --http-port 8123 --max-num-seqs 128 --extra-engine-args '{"min_prefill_tokens": 8000, "max_prefill_delay": 0.3}' > gpurun_out/http_server.log 2>&1 &
SRV=$!
for i in $(seq 1 300); do curl -s localhost:8123/v1/models > /dev/null && break; sleep 1; done
timeout -k 10 600 python tools/loadgen.py --url http://127.0.0.1:8123 --model llama3-8b --isl 3000 --osl 150 --isl-unit chars --concurrency 128 --requests-per-conc 6 --warmup-per-conc 1 --out gpurun_out/http_c128.json > gpurun_out/http_c128.log 2>&1; RC=$?
kill $SRV; wait $SRV 2>/dev/null
tail -4 gpurun_out/http_c128.log
exit $RC
