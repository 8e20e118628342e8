set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
for part in 512 256 1024; do
for v in 1 0 2 3; do
  DX_DECODE_PART=$part DX_DECODE_VARIANT=$v timeout -k 10 120 python tools/microbench.py --what decode > gpurun_out/dec.json 2> gpurun_out/dec.err || { echo FAIL $part $v; tail -20 gpurun_out/dec.err; exit 1; }
  echo "part=$part variant=$v $(python -c "import json;d=json.load(open('gpurun_out/dec.json'));print(' | '.join(f'{k}: {v[\"us\"]}us {v[\"TB/s\"]}TB/s err={v[\"max_err\"]:.3g}' for k,v in d.items()))")" | tee -a gpurun_out/decode_sweep.txt
done
done
