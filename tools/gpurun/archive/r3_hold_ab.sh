#!/bin/bash
# prefill batching hold: closed-loop tok/s and fixed-QPS TTFT at several hold thresholds (one box)
set -o pipefail
mkdir -p gpurun_out
for args in "--min-prefill-tokens 8000 --max-prefill-delay 0.3" "--min-prefill-tokens 5000 --max-prefill-delay 0.2" "--min-prefill-tokens 3000 --max-prefill-delay 0.1" "--min-prefill-tokens 8000 --max-prefill-delay 0.15"; do
  tag=$(echo $args | tr -d ' -' | tr '.' 'p')
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > gpurun_out/hold_$tag.json 2> gpurun_out/hold_$tag.err || { echo "BENCH FAILED $args"; tail -20 gpurun_out/hold_$tag.err; exit 1; }
  echo "$args: $(python -c "import json;d=json.load(open('gpurun_out/hold_$tag.json'));print(d['value'], 'ttft', d['ttft_p50_ms'], '| qps', d['qps'], 'ttft', d['ttft_p50_ms_at_qps'], d['ttft_p99_ms_at_qps'], 'itl', d['itl_p50_ms_at_qps'])")"
done
