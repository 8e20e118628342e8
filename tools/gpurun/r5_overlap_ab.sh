#!/bin/bash
# Mixed-step decode attention on a side stream beside the prefill attention (DX_OVERLAP_DECODE_ATTN=1) vs serial,
# re-measured with the MFMA decode kernel (round 4, VALU decode kernel: no gain, profiles/r3_overlap_probe.txt).
set -o pipefail
mkdir -p gpurun_out/r5ov
O=gpurun_out/r5ov
for ov in 1 0 1 0; do
  DX_OVERLAP_DECODE_ATTN=$ov timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/ov$ov.json 2> $O/ov$ov.err \
    || { tail -20 $O/ov$ov.err; exit 1; }
  echo "overlap=$ov $(tail -1 $O/ov$ov.json | cut -c150-260)"
done
