set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
for v in 4 0; do
  DX_DECODE_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k decode > gpurun_out/t_dec$v.log 2>&1; grep -E "passed|failed|max abs err" gpurun_out/t_dec$v.log | head -8
  echo "variant=$v tests: $(tail -1 gpurun_out/t_dec$v.log)"
  DX_DECODE_VARIANT=$v timeout -k 10 200 python tools/microbench.py --what decode > gpurun_out/dec$v.json 2> gpurun_out/dec$v.err || { echo MB_FAIL; tail gpurun_out/dec$v.err; exit 1; }
  echo "variant=$v $(python -c "import json;d=json.load(open('gpurun_out/dec$v.json'));print(' | '.join(f'{k}: {v[\"us\"]}us {v[\"TB/s\"]}TB/s err={v[\"max_err\"]:.3g}' for k,v in d.items()))")"
done
