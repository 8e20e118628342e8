"""Numerics of the 256x256-tile MFMA GEMM (csrc/kernels/gemm256.hip) against
a plain PyTorch fp32 reference: the plain-store epilogue and the fused SwiGLU
epilogue over 32-row interleaved gate/up weights, at token counts that cover
partial tiles (M not a multiple of 256) and the prefill sizes of the bench."""
import pytest
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.ops import reference as ref


def test_interleave_roundtrip_cpu():
    w = torch.randn(2 * 96, 8)
    wi = ref.interleave_gate_up(w, 32)
    assert torch.equal(ref.deinterleave_gate_up(wi, 32), w)
    gu = torch.randn(5, 2 * 96)
    gi = gu.view(5, 2, 3, 32).permute(0, 2, 1, 3).reshape(5, -1)  # columns in the interleaved order
    assert torch.allclose(ref.silu_and_mul(gi, 32), ref.silu_and_mul(gu), atol=1e-6)
    # the fused path's CPU fallback == unfused reference on de-interleaved weights
    x = torch.randn(7, 8)
    assert torch.allclose(ops.gemm256(x, wi, ops.GEMM256_EPI_SILU).float(),
                          ref.silu_and_mul(ref.linear(x, w)).float(), atol=1e-5)


def _rel(got, want):
    return ((got.float() - want.float()).abs().max() / want.float().abs().max()).item()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 77, 256, 300, 3000, 8192])
@pytest.mark.parametrize("gm", [8, 3, 1008])  # token tiles per L2 band (+1000: one workgroup per tile)
def test_gemm256_store(M, gm):
    torch.manual_seed(M)
    dev = "cuda"
    K, N = 4096, 768
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = (torch.randn(N, K, device=dev) / 64).bfloat16()
    got = ops.gemm256(x, w, group_m=gm)
    want = x.float() @ w.float().t()
    assert _rel(got, want) < 1e-2
    # bias check on a few exact entries: asymmetric operands catch a transposed store
    assert torch.allclose(got[:, :3].float(), want[:, :3], atol=0.02, rtol=0.02)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 128, 300, 3000, 8192])
def test_gemm256_silu(M):
    torch.manual_seed(1 + M)
    dev = "cuda"
    K, F = 4096, 1024
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = (torch.randn(2 * F, K, device=dev) / 64).bfloat16()
    wi = ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous()
    got = ops.gemm256(x, wi, ops.GEMM256_EPI_SILU)
    gu = x.float() @ w.float().t()
    want = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    assert got.shape == (M, F)
    assert _rel(got, want) < 1e-2
    # the interleaved elementwise kernel agrees with the fused epilogue
    gui = ops.gemm256(x, wi)
    assert _rel(ops.silu_and_mul(gui, blk=ops.GEMM256_BLK), want) < 1e-2


@pytest.mark.gpu
def test_gemm256_down_shape_and_strided_x():
    torch.manual_seed(3)
    dev = "cuda"
    M, K, N = 1000, 14336, 512
    big = (torch.rand(M, K + 64, device=dev) * 2 - 1).bfloat16()
    x = big[:, :K]  # row stride K + 64
    w = (torch.randn(N, K, device=dev) / 128).bfloat16()
    got = ops.gemm256(x, w)
    assert _rel(got, x.float() @ w.float().t()) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,epi", [(3000, 6144, 0), (8192, 6144, 0), (2900, 8192, 1), (8192, 4096, 1)])
def test_gemm256_persistent_multi_tile(M, N, epi):
    """More tiles than CUs: each persistent workgroup walks several tiles of its
    XCD's range (uneven per-XCD counts, partial last token tile), and the next
    tile's prologue DMA overlaps the previous tile's stores."""
    torch.manual_seed(M + N)
    dev = "cuda"
    K = 1024
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = (torch.randn(N, K, device=dev) / 32).bfloat16()
    if epi == 0:
        got = ops.gemm256(x, w)
        want = x.float() @ w.float().t()
    else:
        wi = ref.interleave_gate_up(w, ops.GEMM256_BLK).contiguous()
        got = ops.gemm256(x, wi, ops.GEMM256_EPI_SILU)
        gu = x.float() @ w.float().t()
        want = torch.nn.functional.silu(gu[:, :N // 2]) * gu[:, N // 2:]
    assert (-(-M // 256)) * (N // 256) > 256
    assert _rel(got, want) < 1e-2
    # every tile was written: rows / columns at the tile borders match
    for r in (0, 255, 256, M - 1):
        assert torch.allclose(got[r].float(), want[r], atol=0.05, rtol=0.05), r
