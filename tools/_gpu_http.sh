set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
DYN_LOG=warning timeout -k 10 700 python -m dynamo_exp_amd.cli.run in=http out=native --model-path llama3-8b --model-name llama3-8b --http-port 8123 > gpurun_out/http_server.log 2>&1 &
SRV=$!
for i in $(seq 1 240); do curl -s localhost:8123/v1/models > /dev/null && break; sleep 1; done
timeout -k 10 600 python tools/loadgen.py --url http://127.0.0.1:8123 --model llama3-8b --isl 3000 --osl 150 --isl-unit chars --concurrency 1,16,64,128 --requests-per-conc 3 --warmup-per-conc 1 --out gpurun_out/http_sweep.json > gpurun_out/http_sweep.log 2>&1; RC=$?
kill $SRV; wait $SRV 2>/dev/null
cat gpurun_out/http_sweep.log | tail -6
exit $RC
