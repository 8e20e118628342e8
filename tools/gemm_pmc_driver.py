"""Launch driver for rocprofv3 --pmc on the prefill GEMMs: gate_up at M tokens
through the fused SwiGLU gemm256 kernel and through hipBLASLt (+ silu_and_mul),
10 launches each, uniform random operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamo_exp_amd import ops  # noqa: E402
from dynamo_exp_amd.ops import reference as ref  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
H, F = 4096, 14336
x = (torch.rand(M, H, device="cuda") * 2 - 1).bfloat16()
w = ((torch.rand(2 * F, H, device="cuda") * 2 - 1) * H ** -0.5).bfloat16()
wi = ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous()
act = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
gu = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    ops.gemm256(x, wi, ops.GEMM256_EPI_SILU, out=act)
for _ in range(10):
    ops.silu_and_mul(torch.matmul(x, w.t(), out=gu), out=act)
torch.cuda.synchronize()
print("done")
