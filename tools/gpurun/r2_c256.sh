# the decode rank's regime (256 streams per GPU, local prefills): token budget 8192 vs 16384
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c256
for cfg in "8192 8000" "16384 16000" "8192 8000" "16384 16000"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --concurrency 256 --max-batched-tokens $1 --min-prefill-tokens $2 > gpurun_out/c256/b$1.json 2> gpurun_out/c256/b$1.err
  rc=$?; echo "C=256 mbt=$1 mpt=$2 rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/c256/b$1.json'));c=d['config'];print(d['value'], d['ttft_p50_ms'], d['itl_p50_ms'], c['mixed_iters'], c['decode_iters'])")"; [ $rc -eq 0 ] || exit $rc
done
