# prefill batching only under load (--prefill-hold-min-decode): open-loop TTFT and the closed-loop headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hold
for cfg in "8 48" "14 48" "20 48" "closed 48" "closed 64" "20 64"; do
  set -- $cfg
  if [ "$1" = closed ]; then extra=""; else extra="--qps $1"; fi
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 $extra --prefill-hold-min-decode $2 > gpurun_out/hold/$1_$2.json 2> gpurun_out/hold/$1_$2.err
  rc=$?; echo "load=$1 hold_min=$2 rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/hold/$1_$2.json'));print(d['value'], d['ttft_p50_ms'], d['ttft_p99_ms'], d['itl_p50_ms'], d['completed_requests'])")"; [ $rc -eq 0 ] || exit $rc
done
