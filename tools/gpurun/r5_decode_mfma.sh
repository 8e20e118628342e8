#!/bin/bash
# MFMA decode attention (G = 4 / 8, bf16 KV): numerics of both kernels (NaN past each context), then
# throughput MFMA vs VALU over batch / context points at target 512 and 1024 workgroups.
set -o pipefail
mkdir -p gpurun_out/r5mf
O=gpurun_out/r5mf
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kv_fp8.py \
  -m gpu -k "decode" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for MF in 1 0; do
  for W in 512 1024; do
    for H in 32,8 16,2 64,8; do
      DX_DECODE_MFMA=$MF DX_MB_DECODE_ONLY=1 DX_DECODE_WGS=$W timeout -k 10 120 python tools/microbench.py --what attn \
        --heads $H > $O/d_${H/,/_}_w${W}_m$MF.json 2> $O/d.err || { tail -10 $O/d.err; exit 1; }
    done
  done
done
python - <<'PY'
import json
for h in ("32_8", "16_2", "64_8"):
    for W in (512, 1024):
        a = json.load(open(f"gpurun_out/r5mf/d_{h}_w{W}_m1.json")); v = json.load(open(f"gpurun_out/r5mf/d_{h}_w{W}_m0.json"))
        print(h, W, {k.replace("decode_attn_", ""): (v[k]["TB/s"], a[k]["TB/s"]) for k in a})
PY
