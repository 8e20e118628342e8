#!/bin/bash
# MFMA decode attention for every head group (1-16 query heads per KV head): numerics, then MFMA vs VALU at
# G = 1 (8 q / 8 kv) and G = 2 (8 q / 4 kv).
set -o pipefail
mkdir -p gpurun_out/r5mfa
O=gpurun_out/r5mfa
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kv_fp8.py \
  -m gpu -k "decode or fp8" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for MF in 1 0; do
  for H in 8,8 8,4 32,8; do
    DX_DECODE_MFMA=$MF DX_MB_DECODE_ONLY=1 timeout -k 10 120 python tools/microbench.py --what attn \
      --heads $H > $O/d_${H/,/_}_m$MF.json 2> $O/d.err || { tail -10 $O/d.err; exit 1; }
  done
done
python - <<'PY'
import json
for h in ("8_8", "8_4"):
    a = json.load(open(f"gpurun_out/r5mfa/d_{h}_m1.json")); v = json.load(open(f"gpurun_out/r5mfa/d_{h}_m0.json"))
    print(h, {k.replace("decode_attn_", ""): (v[k]["TB/s"], a[k]["TB/s"]) for k in a})
PY
