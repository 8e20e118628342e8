#!/bin/bash
# decode attention with the in-wave lane-group merge: numerics (every G, fp8 KV), then the partition sweep at
# 16 q / 2 KV (one Llama-3-70B TP4 rank) and 32 / 8 (Llama-3-8B) heads.
set -o pipefail
mkdir -p gpurun_out/r5dm
O=gpurun_out/r5dm
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kv_fp8.py \
  -m gpu -k "decode" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for W in 512 1024 2048; do
  for H in 16,2 32,8; do
    DX_MB_DECODE_ONLY=1 DX_DECODE_WGS=$W timeout -k 10 120 python tools/microbench.py --what attn --heads $H \
      > $O/dattn_${H/,/_}_w$W.json 2> $O/dattn.err || { tail -10 $O/dattn.err; exit 1; }
  done
done
python - <<'PY'
import json
for h in ("16_2", "32_8"):
    for W in (512, 1024, 2048):
        d = json.load(open(f"gpurun_out/r5dm/dattn_{h}_w{W}.json"))
        print(h, W, {k: (v["TB/s"], v["parts"]) for k, v in d.items()})
PY
