#!/bin/bash
# decode attention after the in-wave merge: the flash-decoding target workgroup count (ops.DECODE_TARGET_WGS,
# env DX_DECODE_WGS) swept over batch / context points for 32 q / 8 kv (Llama-3-8B), 16 / 2 (one 70B TP4 rank),
# 64 / 8 (70B TP1) and 8 / 8 (G = 1).
set -o pipefail
mkdir -p gpurun_out/r5dw
O=gpurun_out/r5dw
for W in 256 512 1024 2048; do
  for H in 32,8 16,2 64,8 8,8; do
    DX_MB_DECODE_ONLY=1 DX_DECODE_WGS=$W timeout -k 10 120 python tools/microbench.py --what attn --heads $H \
      > $O/dattn_${H/,/_}_w$W.json 2> $O/dattn.err || { tail -10 $O/dattn.err; exit 1; }
  done
done
python - <<'PY'
import json
for h in ("32_8", "16_2", "64_8", "8_8"):
    rows = {W: json.load(open(f"gpurun_out/r5dw/dattn_{h}_w{W}.json")) for W in (256, 512, 1024, 2048)}
    for k in rows[512]:
        print(h, k, {W: (rows[W][k]["TB/s"], rows[W][k]["parts"]) for W in rows})
PY
