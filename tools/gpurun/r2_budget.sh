# token budget aligned to whole prompts (no small tail chunk): bench.py --max-batched-tokens B --min-prefill-tokens H
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/budget
for cfg in "8192 8000" "9216 8000" "9216 9000" "6272 6000" "8192 8000"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --max-batched-tokens $1 --min-prefill-tokens $2 > gpurun_out/budget/b$1_$2.json 2> gpurun_out/budget/b$1_$2.err
  rc=$?; echo "mbt=$1 mpt=$2 rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/budget/b$1_$2.json'));c=d['config'];print(d['value'], d['ttft_p50_ms'], d['itl_p50_ms'], c['mixed_iters'], c['decode_iters'])")"; [ $rc -eq 0 ] || exit $rc
done
