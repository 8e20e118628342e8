set -o pipefail
mkdir -p gpurun_out
for cfg in "8000 0.5 8192" "12000 0.5 16384" "16000 1.0 16384"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --min-prefill-tokens $1 --max-prefill-delay $2 --max-batched-tokens $3 --verbose > gpurun_out/pb2_$1.json 2> gpurun_out/pb2_$1.err || { echo BENCH_FAIL $cfg; tail -20 gpurun_out/pb2_$1.err; exit 1; }
  echo "$cfg $(cat gpurun_out/pb2_$1.json)"
  grep "engine timing" gpurun_out/pb2_$1.err | tail -1
done
