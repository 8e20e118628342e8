set -o pipefail
mkdir -p gpurun_out
for ov in 1 0 1; do
DX_OVERLAP_DECODE_ATTN=$ov timeout -k 10 600 python -u bench.py > gpurun_out/bench_ov$ov.json 2> gpurun_out/bench_ov$ov.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_ov$ov.json'));print('overlap=$ov', d['value'], d['ttft_p50_ms'], d['config']['itl_p50_ms'])"
done
