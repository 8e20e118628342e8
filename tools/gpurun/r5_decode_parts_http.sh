#!/bin/bash
# (a) decode attention at one Llama-3-70B TP4 rank's 16 q / 2 KV heads vs the partition count (DX_DECODE_WGS:
#     target workgroups per launch); (b) the HTTP-vs-bench comparison with the staggered loadgen.
set -o pipefail
mkdir -p gpurun_out/r5dp
O=gpurun_out/r5dp
for W in 256 512 1024 2048; do
  DX_MB_DECODE_ONLY=1 DX_DECODE_WGS=$W timeout -k 10 120 python tools/microbench.py --what attn --heads 16,2 \
    > $O/dattn_16_2_w$W.json 2> $O/dattn_w$W.err || { tail -10 $O/dattn_w$W.err; exit 1; }
  DX_MB_DECODE_ONLY=1 DX_DECODE_WGS=$W timeout -k 10 120 python tools/microbench.py --what attn --heads 32,8 \
    > $O/dattn_32_8_w$W.json 2> $O/dattn8_w$W.err || { tail -10 $O/dattn8_w$W.err; exit 1; }
done
python - <<'PY'
import json
for h in ("16_2", "32_8"):
    for W in (256, 512, 1024, 2048):
        d = json.load(open(f"gpurun_out/r5dp/dattn_{h}_w{W}.json"))
        print(h, W, {k: (v["TB/s"], v["parts"]) for k, v in d.items()})
PY
bash tools/gpurun/r5_http_vs_bench.sh
