"""Launch driver for rocprofv3 --pmc on the folded-norm kernels at a mixed
step's size (T = 8192 tokens, Llama-3-8B layer shapes): row_rrms, the fused
SwiGLU GEMM with row scales (EPI_SILU_RS) next to the plain SwiGLU epilogue,
the o-projection as hipBLASLt addmm_ (beta = 1) next to a plain matmul, and
rope_cache with and without a row scale; 10 launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.ops import reference as ref  # noqa: E402

T, H, F, Hq, Hkv, D, BS = 8192, 4096, 14336, 32, 8, 128, 64
dev = "cuda"
res = (torch.randn(T, H, device=dev)).bfloat16()
w = ((torch.rand(2 * F, H, device=dev) * 2 - 1) * H ** -0.5).bfloat16()
wi = ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous()
wo = ((torch.rand(H, H, device=dev) * 2 - 1) * H ** -0.5).bfloat16()
attn = (torch.rand(T, H, device=dev) * 2 - 1).bfloat16()
act = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
rs = torch.empty(T, device=dev, dtype=torch.float32)
qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev).bfloat16()
pos = torch.arange(T, device=dev) % 4096
cos_sin = ref.rope_cos_sin(D, 8192, 500000.0).to(dev)
nb = T // BS + 2
kc = torch.zeros(nb, Hkv, BS, D, device=dev).bfloat16()
vc = torch.zeros_like(kc)
slots = torch.arange(T, device=dev, dtype=torch.int64)
for _ in range(10):
    ops.row_rrms(res, 1e-5, out=rs)
order = [True, False] if os.environ.get("DX_FOLD_PMC_ORDER", "rs_first") == "rs_first" else [False, True]
for scaled in order + order:  # each variant twice, interleaved: clock ramps hit both alike
    for _ in range(5):
        ops.gemm256(res, wi, ops.GEMM256_EPI_SILU, out=act, row_scale=rs if scaled else None)
out = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
for _ in range(10):
    torch.matmul(attn, wo.t(), out=out)
for _ in range(10):
    out.addmm_(attn, wo.t())
for _ in range(10):
    ops.rope_cache(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, D, BS, row_scale=rs)
for _ in range(10):
    ops.rope_cache(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, D, BS)
torch.cuda.synchronize()
print("done")
