set -o pipefail
mkdir -p gpurun_out
for k in 1 2 4; do
  DX_MULTI_STEP=$k timeout -k 10 300 python -u bench.py > gpurun_out/ms2_$k.json 2> gpurun_out/ms2_$k.err || { echo BENCH_FAIL $k; tail -20 gpurun_out/ms2_$k.err; exit 1; }
  echo "ms=$k $(cut -c1-60 gpurun_out/ms2_$k.json | head -c 0)$(python -c "import json;d=json.load(open('gpurun_out/ms2_$k.json'));print(d['value'],d['ttft_p50_ms'],d['config']['itl_p50_ms'],d['config']['decode_steps'],d['config']['mixed_steps'])")"
done
