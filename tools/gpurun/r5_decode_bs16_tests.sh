#!/bin/bash
# block size 16 (the vLLM default): the MFMA decode kernel with two blocks per 32-token chunk -- numerics of both
# kernels, then MFMA vs VALU throughput
set -o pipefail
mkdir -p gpurun_out/r5bs16
O=gpurun_out/r5bs16
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kv_fp8.py -m gpu -k "decode or fp8" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for MF in 1 0; do
  for H in 32,8 16,2; do
    DX_MB_BLOCK=16 DX_DECODE_MFMA=$MF DX_MB_DECODE_ONLY=1 timeout -k 10 120 python tools/microbench.py --what attn \
      --heads $H > $O/d_${H/,/_}_m$MF.json 2> $O/d.err || { tail -10 $O/d.err; exit 1; }
  done
done
python - <<'PY'
import json
for h in ("32_8", "16_2"):
    a = json.load(open(f"gpurun_out/r5bs16/d_{h}_m1.json")); v = json.load(open(f"gpurun_out/r5bs16/d_{h}_m0.json"))
    print(h, {k.replace("decode_attn_", ""): (v[k]["TB/s"], a[k]["TB/s"]) for k in a})
PY
