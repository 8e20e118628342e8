set -o pipefail
mkdir -p gpurun_out
for cfg in "0 0" "6000 0.15" "8000 0.3" "4500 0.1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --min-prefill-tokens $1 --max-prefill-delay $2 > gpurun_out/pb_$1.json 2> gpurun_out/pb_$1.err || { echo BENCH_FAIL $cfg; tail -20 gpurun_out/pb_$1.err; exit 1; }
  echo "$cfg $(cat gpurun_out/pb_$1.json)"
done
