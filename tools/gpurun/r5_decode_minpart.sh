#!/bin/bash
# decode attention (MFMA kernel, bf16): minimum tokens per flash-decoding partition (DX_DECODE_MIN_PART) at
# target 512 workgroups -- the small-batch points are where the cap binds.
set -o pipefail
mkdir -p gpurun_out/r5mp
O=gpurun_out/r5mp
for MP in 256 128 64; do
  for H in 32,8 16,2; do
    DX_DECODE_MIN_PART=$MP DX_MB_DECODE_ONLY=1 timeout -k 10 120 python tools/microbench.py --what attn --heads $H \
      > $O/d_${H/,/_}_mp$MP.json 2> $O/d.err || { tail -10 $O/d.err; exit 1; }
  done
done
python - <<'PY'
import json
for h in ("32_8", "16_2"):
    rows = {mp: json.load(open(f"gpurun_out/r5mp/d_{h}_mp{mp}.json")) for mp in (256, 128, 64)}
    for k in rows[256]:
        print(h, k, {mp: (rows[mp][k]["us"], rows[mp][k]["parts"]) for mp in rows})
PY
