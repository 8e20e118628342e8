"""Engine ops.  GPU tensors run the hand-written gfx950 HIP kernels
(``_C_kernels``); CPU tensors run the fp32 PyTorch references in
:mod:`.reference` (CPU CI only).  A GPU call never falls back: if the kernel
extension is missing it raises.

Kernel layouts (see the .hip sources for the design notes):
  * paged KV cache per layer: K, V = [num_blocks, Hkv, block_size, D] bf16
  * fused QKV activations: [T, (Hq + 2 Hkv) * D] bf16, Q/K rotated in place
"""
from __future__ import annotations

import math
import os

from typing import NamedTuple

import torch

from .. import _native
from . import reference as ref

__all__ = [
    "rmsnorm",
    "add_rmsnorm",
    "SplitK",
    "splitk_reduce",
    "rope_cache",
    "kv_write",
    "silu_and_mul",
    "embedding",
    "decode_attention",
    "prefill_attention",
    "prefill_work_list",
    "fp8_scratch_plan",
    "sample",
    "apply_penalties",
    "kv_copy_blocks",
    "DECODE_TARGET_WGS",
    "DECODE_MIN_PART",
    "decode_num_parts",
    "rmsnorm_quant",
    "silu_mul_quant",
    "quant_rows",
    "fp8_linear",
]

# decode attention partitioning (decode_num_parts): aim for this many
# workgroups per launch, never split a context into parts shorter than
# DECODE_MIN_PART tokens.  512 since the round-5 in-wave merge cut the
# per-workgroup epilogue: best or within 3 % of best at every batch / context /
# head layout swept (profiles/r5_decode_wgs_sweep.txt; 2048 was the round-1
# optimum with the 64-state LDS merge)
DECODE_TARGET_WGS = int(os.environ.get("DX_DECODE_WGS", "512"))
DECODE_MIN_PART = int(os.environ.get("DX_DECODE_MIN_PART", "256"))


def _k():
    return _native.kernels()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _chk(t: torch.Tensor, dtype=None, name="tensor"):
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.stride(-1) != 1:
        raise ValueError(f"{name}: last dim must be contiguous")


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None) -> torch.Tensor:
    if not x.is_cuda:
        r = ref.rmsnorm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    _chk(x, torch.bfloat16, "x")
    rows, hidden = x.shape
    out = torch.empty_like(x) if out is None else out
    _k().rmsnorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), rows, hidden, x.stride(0), out.stride(0), float(eps), _stream())
    return out


class SplitK(NamedTuple):
    """A decode projection's output still as split-K partials (dstream_linear
    with partial=True): `splits` fp32 slabs of [bm][n] rows in the per-stream
    workspace, slice s / row m at slabs[(s * bm + m) * n].  Consumed once, by
    the very next kernel on the stream (add_rmsnorm sums them itself) before
    any other small-M GEMM reuses the workspace."""
    slabs: torch.Tensor
    splits: int
    bm: int
    m: int
    n: int
    dtype: torch.dtype

    @property
    def shape(self):
        return (self.m, self.n)

    @property
    def is_cuda(self) -> bool:
        return True


def splitk_reduce(p: SplitK, out: torch.Tensor | None = None) -> torch.Tensor:
    """The bf16 [m, n] tensor of a SplitK (the reduction kernel dstream_linear
    would have launched), for consumers that need a plain tensor."""
    out = torch.empty((p.m, p.n), dtype=p.dtype, device=p.slabs.device) if out is None else out
    _k().splitk_reduce(out.data_ptr(), out.stride(0), p.slabs.data_ptr(), p.m, p.n, p.bm, p.splits, _stream())
    return out


def add_rmsnorm(x, residual: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    """residual += x (in place); return rmsnorm(residual) * w (into `out`, may alias x).
    x may be a SplitK: its partials are summed inside the norm kernel (bit-equal
    to reducing first); then `out` must be a separate [m, hidden] tensor or None."""
    if isinstance(x, SplitK):
        out = torch.empty((x.m, x.n), dtype=residual.dtype, device=residual.device) if out is None else out
        _k().add_rmsnorm_slabs(out.data_ptr(), x.slabs.data_ptr(), x.splits, x.bm, residual.data_ptr(), w.data_ptr(),
                               x.m, x.n, out.stride(0), residual.stride(0), float(eps), _stream())
        return out
    if not x.is_cuda:
        r = ref.add_rmsnorm(x, residual, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    _chk(x, torch.bfloat16, "x")
    rows, hidden = x.shape
    out = torch.empty_like(x) if out is None else out
    _k().add_rmsnorm(out.data_ptr(), x.data_ptr(), residual.data_ptr(), w.data_ptr(), rows, hidden, x.stride(0),
                     out.stride(0), residual.stride(0), float(eps), _stream())
    return out


KV_FP8 = torch.float8_e4m3fn  # KV cache dtype of the fp8 cache (kv_cache_dtype="fp8")


def _kv_fp8(k_cache) -> bool:
    return k_cache.dtype == KV_FP8


def rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, n_q, n_kv, head_dim, block_size, rotate_q=True,
               kv_scales=(1.0, 1.0), out: torch.Tensor | None = None, row_scale: torch.Tensor | None = None):
    """Rotary on Q/K in place + K/V written to the paged cache (bf16, or e4m3fn
    of x / scale with per-tensor `kv_scales` for an fp8 cache).  qkv may be a
    SplitK (the QKV projection's partials): the kernel sums them and writes the
    whole row (rotated Q / K, V) into `out` [T, row] bf16, which it returns.
    row_scale [T] fp32: a deferred RMSNorm of the projection's input rows
    (`row_rrms`; the norm weight folded into the weights): Q, K, V are scaled
    by it first (Q in the row, K / V in the cache)."""
    if row_scale is not None:
        assert not isinstance(qkv, SplitK), "row_scale needs a finished projection row"
        assert row_scale.dtype == torch.float32 and row_scale.shape == (qkv.shape[0],)
        if not qkv.is_cuda:
            qkv.copy_((qkv.float() * row_scale[:, None]).to(qkv.dtype))
            row_scale = None
    if isinstance(qkv, SplitK):
        T, row = qkv.m, qkv.n
        out = torch.empty((T, row), dtype=qkv.dtype, device=qkv.slabs.device) if out is None else out
        assert out.shape == (T, row) and out.stride(1) == 1 and row == (n_q + 2 * n_kv) * head_dim
        slabs, splits, bm, qkv = qkv.slabs.data_ptr(), qkv.splits, qkv.bm, out
    else:
        slabs, splits, bm = 0, 0, 0
    if not qkv.is_cuda:
        return ref.rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, n_q, n_kv, head_dim, block_size,
                              rotate_q, kv_scales)
    _chk(qkv, torch.bfloat16, "qkv")
    assert cos_sin.dtype == torch.float32 and cos_sin.shape[1] == head_dim
    assert slot_mapping is None or slot_mapping.dtype == torch.int64
    assert k_cache.dtype in (torch.bfloat16, KV_FP8) and v_cache.dtype == k_cache.dtype
    T = qkv.shape[0]
    _k().rope_cache(qkv.data_ptr(), qkv.stride(0), positions.data_ptr(), int(positions.dtype == torch.int64),
                    cos_sin.data_ptr(), 0 if slot_mapping is None else slot_mapping.data_ptr(), k_cache.data_ptr(),
                    v_cache.data_ptr(), T, n_q, n_kv, head_dim, block_size, int(rotate_q), int(_kv_fp8(k_cache)),
                    float(kv_scales[0]), float(kv_scales[1]), slabs, splits, bm, _stream(),
                    0 if row_scale is None else row_scale.data_ptr())
    return qkv


def row_rrms(x: torch.Tensor, eps: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """1 / rms of each row of x [T, H] bf16 -> [T] fp32: the scale of an RMSNorm
    folded into its consumers (models/llama.py)."""
    if not x.is_cuda:
        r = torch.rsqrt(x.float().pow(2).mean(-1) + eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    _chk(x, torch.bfloat16, "x")
    rows, hidden = x.shape
    out = torch.empty(rows, dtype=torch.float32, device=x.device) if out is None else out
    assert out.dtype == torch.float32 and out.shape == (rows,) and out.is_contiguous()
    _k().row_rrms(out.data_ptr(), x.data_ptr(), rows, hidden, x.stride(0), float(eps), _stream())
    return out


def kv_write(k, v, slot_mapping, k_cache, v_cache, block_size, kv_scales=(1.0, 1.0)):
    """k, v: [T, Hkv, D] views with equal token stride."""
    if not k.is_cuda or _kv_fp8(k_cache):  # fp8 caches: the torch path (receive-path tests only)
        return ref.write_kv(k, v, slot_mapping, k_cache, v_cache, block_size, kv_scales)
    assert k.stride(0) == v.stride(0)
    T, hkv, hd = k.shape
    _k().kv_write(k.data_ptr(), v.data_ptr(), k.stride(0), slot_mapping.data_ptr(), k_cache.data_ptr(),
                  v_cache.data_ptr(), T, hkv, hd, block_size, _stream())


def silu_and_mul(gate_up: torch.Tensor, out: torch.Tensor | None = None, blk: int = 0) -> torch.Tensor:
    """silu(gate) * up; blk > 0: gate / up columns interleaved in blocks of blk."""
    if not gate_up.is_cuda:
        r = ref.silu_and_mul(gate_up, blk)
        if out is not None:
            out.copy_(r)
            return out
        return r
    _chk(gate_up, torch.bfloat16, "gate_up")
    T, f2 = gate_up.shape
    f = f2 // 2
    out = torch.empty((T, f), dtype=gate_up.dtype, device=gate_up.device) if out is None else out
    _k().silu_and_mul(out.data_ptr(), gate_up.data_ptr(), T, f, gate_up.stride(0), out.stride(0), blk, _stream())
    return out


# ---------------------------------------------------------------- large-M GEMM
GEMM256_EPI_STORE, GEMM256_EPI_SILU, GEMM256_EPI_SILU_RS = 0, 1, 2
GEMM256_BLK = 32  # gate / up interleave of the fused SwiGLU epilogue


def gemm256_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether the 256x256-tile MFMA GEMM (csrc/kernels/gemm256.hip) takes
    this x [M, K] . w [N, K]^T."""
    M, K = x.shape
    N = w.shape[0]
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[1] == K
            and N % 256 == 0 and K % 128 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0 and w.is_contiguous() and w.data_ptr() % 16 == 0 and N * K < 2 ** 31
            and 256 * x.stride(0) < 2 ** 31)


def gemm256(x: torch.Tensor, w: torch.Tensor, epi: int = GEMM256_EPI_STORE, out: torch.Tensor | None = None,
            group_m: int = 8, row_scale: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w.T (epi 0) or the fused SwiGLU y = silu(x @ g.T) * (x @ u.T)
    over 32-row interleaved gate/up weights (epi 1, y has N/2 columns), on the
    hand-written 256x256-tile MFMA kernel; group_m = token tiles per L2 band.
    row_scale [M] fp32 (SwiGLU only): the rows' deferred RMSNorm scale, applied
    to g and u before the activation (epi 2)."""
    if row_scale is not None:
        if epi != GEMM256_EPI_SILU:
            raise ValueError("gemm256: row_scale needs the SwiGLU epilogue")
        assert row_scale.dtype == torch.float32 and row_scale.shape == (x.shape[0],) and row_scale.is_contiguous()
        epi = GEMM256_EPI_SILU_RS
    if not x.is_cuda:
        y = ref.linear(x, w)
        if epi == GEMM256_EPI_SILU_RS:
            y = (y.float() * row_scale[:, None]).to(y.dtype)
        y = ref.silu_and_mul(y, GEMM256_BLK) if epi in (GEMM256_EPI_SILU, GEMM256_EPI_SILU_RS) else y
        if out is not None:
            out.copy_(y)
            return out
        return y
    if not gemm256_ok(x, w):
        raise ValueError(f"gemm256: unsupported operands x{tuple(x.shape)} w{tuple(w.shape)}")
    M, K = x.shape
    N = w.shape[0]
    cols = N // 2 if epi in (GEMM256_EPI_SILU, GEMM256_EPI_SILU_RS) else N
    out = torch.empty((M, cols), dtype=x.dtype, device=x.device) if out is None else out
    if out.shape != (M, cols) or out.stride(1) != 1 or out.stride(0) % 4 or out.data_ptr() % 8:
        raise ValueError("gemm256: bad out tensor")
    _k().gemm256(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), M, N, K, epi, group_m,
                 _stream(), 0 if row_scale is None else row_scale.data_ptr())
    return out


# ---------------------------------------------------------------- small-M GEMM
SKINNY_MAX_M = 256
# (device, stream) -> (slabs fp32, tickets int32).  Keyed by stream: two
# launches in flight on different streams must never share split-K slabs or
# tickets (the kernel's last-arriver reduction would mix their partial sums).
# A graph captured on a stream keeps that stream's workspace alive here.
_SKINNY_WS: dict = {}
SKINNY_SLAB_FLOATS = 8 << 20  # 32 MiB of split-K slabs per (device, stream)
SKINNY_TICKETS = 1 << 16


def _skinny_ws(device, stream: int):
    key = (device, stream)
    ws = _SKINNY_WS.get(key)
    if ws is None:
        ws = (torch.empty(SKINNY_SLAB_FLOATS, dtype=torch.float32, device=device),
              torch.zeros(SKINNY_TICKETS, dtype=torch.int32, device=device))
        _SKINNY_WS[key] = ws
    return ws


def skinny_configs(M: int, N: int, K: int) -> list[tuple[int, int, int]]:
    """Valid (bn, bm, splits) launch configurations of the small-M GEMM."""
    out = []
    if not (1 <= M <= SKINNY_MAX_M) or K % 256:
        return out
    mp = -(-M // 32) * 32  # wide kernel: one workgroup covers all rows, K split over workgroups only
    if N % 128 == 0:
        for s in (1, 2, 4, 8):
            if K % (s * (128 if mp <= 128 else 64)) == 0 and (s == 1 or (s * mp * N <= SKINNY_SLAB_FLOATS and N // 128 <= SKINNY_TICKETS)):
                out.append((128, mp, s))
    for bn in (32, 64):
        if N % bn:
            continue
        for bm in (32, 64):
            mp = -(-M // bm) * bm
            for s in (1, 2, 4, 8):
                if K % (s * 256):
                    continue
                if s > 1 and (s * mp * N > SKINNY_SLAB_FLOATS or (N // bn) * (mp // bm) > SKINNY_TICKETS):
                    continue
                out.append((bn, bm, s))
    return out


# the stage ring of an LDS-staged decode GEMM must fit one CU's LDS
STREAM_LDS = 160 * 1024


DSTREAM = "ds"  # config tag of the deep-stream kernel: ("ds", waves, r, t, dw, dx, splits)
# (nw, r, t) instantiated in csrc/kernels/dstream_gemm.hip; (dw, dx) in DSTREAM_DEPTHS
DSTREAM_SHAPES = {(4, 1, 2), (4, 1, 4), (4, 1, 8), (4, 1, 16), (4, 2, 2), (4, 2, 4), (4, 2, 8), (4, 2, 16),
                  (8, 1, 2), (8, 1, 4), (8, 1, 8), (8, 1, 16), (8, 2, 2), (8, 2, 4), (8, 2, 8)} | {
    # 3 / 6 / 7-wave row tiles: grids of exactly 256 workgroups for N = 6144 (qkv) and 28672 (gate_up)
    (nw, r, t) for nw in (3, 6, 7) for r, t in ((1, 4), (1, 8), (1, 16), (2, 4), (2, 8))}
DSTREAM_DEPTHS = ((4, 2), (4, 4), (8, 2), (8, 4))


def _dstream_ok(M, N, K, nw, r, t, dw, dx, splits) -> bool:
    ke = 64  # k per 128-B step
    nk = K // ke // max(1, splits)
    return (1 <= M <= 16 * t and t * 16 <= SKINNY_MAX_M and (nw, r, t) in DSTREAM_SHAPES and (dw, dx) in DSTREAM_DEPTHS
            and dx * 16 * t * 128 + 1040 <= STREAM_LDS and not (nw == 4 and r == 2 and t == 16 and dw == 8 and dx == 4)
            and N % (nw * 16 * r) == 0 and K % (ke * splits) == 0 and nk >= dw and nk % dw == 0
            and (splits == 1 or (splits * 16 * t * N <= SKINNY_SLAB_FLOATS and N // (nw * 16 * r) <= SKINNY_TICKETS)))


def dstream_configs(M: int, N: int, K: int, max_grid: int = 2048) -> list[tuple]:
    """Launch configurations of the deep-stream decode GEMM
    (csrc/kernels/dstream_gemm.hip): the smallest token tile holding M,
    4 / 8 waves x 1-2 16-row blocks, weight / x ring depths, split-K; grids
    of 128 .. max_grid workgroups (fewer leave CUs without a weight stream)."""
    out = []
    if not 1 <= M <= SKINNY_MAX_M or K % 64:
        return out
    t = next(tt for tt in (2, 4, 8, 16) if 16 * tt >= M)
    for nw in (3, 4, 6, 7, 8):
        for r in (1, 2):
            for dw, dx in DSTREAM_DEPTHS:
                for s in (1, 2, 4, 8):
                    if not _dstream_ok(M, N, K, nw, r, t, dw, dx, s):
                        continue
                    grid = N // (nw * 16 * r) * s
                    if 128 <= grid <= max_grid:
                        out.append((DSTREAM, nw, r, t, dw, dx, s))
    return out


def dstream_tune_configs(M: int, N: int, K: int) -> list[tuple]:
    """The subset of dstream_configs the engine's warm-up tuner times: from
    M 16 up, grids of 192-1024 workgroups (every CU streaming, at most four
    workgroups per CU) -- DX_DSTREAM=0 leaves the kernel out."""
    if M < 16 or os.environ.get("DX_DSTREAM", "1") == "0":
        return []
    return [c for c in dstream_configs(M, N, K) if 192 <= N // (c[1] * 16 * c[2]) * c[6] <= 1024]


def dstream_linear(x: torch.Tensor, w: torch.Tensor, cfg: tuple, out: torch.Tensor | None = None,
                   partial: bool = False, silu: bool = False):
    """y = x @ w.T on the deep-stream kernel; cfg = ("ds", waves, r, t, dw, dx, splits).
    partial=True with splits > 1: return the split-K partials as a SplitK
    (no reduction launch) for a consumer that sums them (add_rmsnorm).
    silu=True: w is the MLP's gate_up with gate / up rows interleaved in
    blocks of 32 (models/llama.py enable_fused_mlp) and the result is the
    SwiGLU activation [M, N / 2] (needs r == 2)."""
    _, nw, r, t, dw, dx, splits = cfg
    M, K = x.shape
    N = w.shape[0]
    if silu:
        if not x.is_cuda:
            return silu_and_mul(ref.linear(x, w), blk=GEMM256_BLK)
        if r != 2 or N % 64 or partial:
            raise ValueError(f"dstream_linear(silu): config {cfg} / N={N} cannot pair gate and up blocks")
    if x.stride(1) != 1 or w.shape[1] != K or not w.is_contiguous():
        raise ValueError("dstream_linear: x rows and w must be unit-stride with matching K")
    if x.data_ptr() % 16 or w.data_ptr() % 16 or x.stride(0) % 8:
        raise ValueError("dstream_linear: x / w must be 16-byte aligned")
    if not _dstream_ok(M, N, K, nw, r, t, dw, dx, splits):
        raise ValueError(f"dstream_linear: config {cfg} invalid for M={M} N={N} K={K}")
    st = _stream()
    slabs, tickets = _skinny_ws(x.device, st)
    if silu:
        out = torch.empty((M, N // 2), dtype=x.dtype, device=x.device) if out is None else out
        if (out.shape != (M, N // 2) or out.stride(1) != 1 or out.dtype != x.dtype or out.stride(0) % 8
                or out.data_ptr() % 16):
            raise ValueError("dstream_linear(silu): bad out tensor")
        _k().dstream_gemm(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), slabs.data_ptr(),
                          tickets.data_ptr(), M, N, K, nw, r, t, dw, dx, splits, 2, st)
        return out
    if partial and splits > 1 and out is None:
        _k().dstream_gemm(0, N, x.data_ptr(), x.stride(0), w.data_ptr(), slabs.data_ptr(), tickets.data_ptr(), M, N, K,
                          nw, r, t, dw, dx, splits, 1, st)
        return SplitK(slabs, splits, 16 * t, M, N, x.dtype)
    out = torch.empty((M, N), dtype=x.dtype, device=x.device) if out is None else out
    if out.shape != (M, N) or out.stride(1) != 1 or out.dtype != x.dtype or out.stride(0) % 4 or out.data_ptr() % 8:
        raise ValueError("dstream_linear: bad out tensor")
    _k().dstream_gemm(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), slabs.data_ptr(),
                      tickets.data_ptr(), M, N, K, nw, r, t, dw, dx, splits, 0, st)
    return out


def skinny_linear(x: torch.Tensor, w: torch.Tensor, cfg: tuple, out: torch.Tensor | None = None,
                  partial: bool = False):
    """y = x @ w.T for decode-sized x (M <= 256 rows) on the hand-written MFMA
    kernels (csrc/kernels/skinny_gemm.hip; cfg = (bn, bm, splits), or
    csrc/kernels/dstream_gemm.hip; cfg = ("ds", waves, r, t, dw, dx, splits)) from
    the model's tuning pass (models/llama.py tune_gemms)."""
    if not x.is_cuda:
        return ref.linear(x, w)
    _chk(w, torch.bfloat16, "w")
    if cfg[0] == DSTREAM:
        return dstream_linear(x, w, cfg, out, partial=partial)
    M, K = x.shape
    N = w.shape[0]
    if x.stride(1) != 1 or w.shape[1] != K or not w.is_contiguous():
        raise ValueError("skinny_linear: x rows and w must be unit-stride with matching K")
    bn, bm, splits = cfg
    if x.data_ptr() % 16 or w.data_ptr() % 16 or x.stride(0) % 8:
        raise ValueError("skinny_linear: x / w must be 16-byte aligned")
    kq = (128 if bm <= 128 else 64) if bn == 128 else 256
    if not (1 <= M <= SKINNY_MAX_M) or N % bn or K % (splits * kq) or (bn == 128 and bm != -(-M // 32) * 32) or (
            splits > 1 and splits * (-(-M // bm) * bm) * N > SKINNY_SLAB_FLOATS):
        raise ValueError(f"skinny_linear: config {cfg} invalid for M={M} N={N} K={K}")
    out = torch.empty((M, N), dtype=x.dtype, device=x.device) if out is None else out
    if out.shape != (M, N) or out.stride(1) != 1 or out.dtype != x.dtype:
        raise ValueError("skinny_linear: bad out tensor")
    st = _stream()
    slabs, tickets = _skinny_ws(x.device, st)
    _k().skinny_gemm(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), slabs.data_ptr(),
                     tickets.data_ptr(), M, N, K, bn, bm, splits, st)
    return out


# ---------------------------------------------------------------- fp8 (w8a8)
FP8 = torch.float8_e4m3fn


def _fp8_out(rows: int, cols: int, device):
    return torch.empty((rows, cols), dtype=FP8, device=device), torch.empty((rows, 1), dtype=torch.float32, device=device)


def rmsnorm_quant(x: torch.Tensor, residual: torch.Tensor | None, w: torch.Tensor, eps: float):
    """[residual += x (in place);] y = rmsnorm(residual or x) * w -> (e4m3 rows, per-row scales [T, 1])."""
    if not x.is_cuda:
        y = ref.add_rmsnorm(x, residual, w, eps) if residual is not None else ref.rmsnorm(x, w, eps)
        return ref.quant_fp8_rows(y.to(torch.bfloat16))
    _chk(x, torch.bfloat16, "x")
    rows, hidden = x.shape
    q, s = _fp8_out(rows, hidden, x.device)
    _k().rmsnorm_quant(q.data_ptr(), s.data_ptr(), x.data_ptr(), 0 if residual is None else residual.data_ptr(),
                       w.data_ptr(), rows, hidden, x.stride(0), 0 if residual is None else residual.stride(0),
                       float(eps), _stream())
    return q, s


def silu_mul_quant(gate_up: torch.Tensor):
    """silu(gate) * up -> (e4m3 rows [T, F], per-row scales [T, 1])."""
    if not gate_up.is_cuda:
        return ref.quant_fp8_rows(ref.silu_and_mul(gate_up).float())
    _chk(gate_up, torch.bfloat16, "gate_up")
    T, f2 = gate_up.shape
    q, s = _fp8_out(T, f2 // 2, gate_up.device)
    _k().silu_mul_quant(q.data_ptr(), s.data_ptr(), gate_up.data_ptr(), T, f2 // 2, gate_up.stride(0), _stream())
    return q, s


def quant_rows(x: torch.Tensor):
    """bf16 rows -> (e4m3 rows, per-row scales [T, 1])."""
    if not x.is_cuda:
        return ref.quant_fp8_rows(x)
    _chk(x, torch.bfloat16, "x")
    rows, cols = x.shape
    assert x.stride(1) == 1
    q, s = _fp8_out(rows, cols, x.device)
    _k().quant_rows(q.data_ptr(), s.data_ptr(), x.data_ptr(), rows, cols, x.stride(0), _stream())
    return q, s


def fp8_linear(x8: torch.Tensor, sx: torch.Tensor, w8: torch.Tensor, sw: torch.Tensor) -> torch.Tensor:
    """(x8 * sx) @ (w8 * sw)^T -> bf16 (row-wise token scales x column-wise
    channel scales; w8: [N, K] e4m3, sw: [1, N]) through hipBLASLt's fp8
    kernels (round 5's fp8 deep-stream form was removed: its first launch
    faulted, cause unknown -- profiles/r5_dstream_fp8_fault.txt)."""
    if not x8.is_cuda:
        return ref.fp8_linear(x8, sx, w8, sw)
    return torch._scaled_mm(x8, w8.t(), scale_a=sx, scale_b=sw, out_dtype=torch.bfloat16)


def embedding(ids: torch.Tensor, table: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    if not ids.is_cuda:
        r = ref.embedding(ids, table)
        if out is not None:
            out.copy_(r)
            return out
        return r
    T = ids.shape[0]
    V, H = table.shape
    out = torch.empty((T, H), dtype=table.dtype, device=table.device) if out is None else out
    _k().embedding(out.data_ptr(), table.data_ptr(), ids.data_ptr(), int(ids.dtype == torch.int64), T, H, V, _stream())
    return out


def decode_num_parts(batch: int, n_kv_heads: int, max_ctx: int) -> int:
    """Balanced flash-decoding partitions per sequence for a decode launch of
    `batch` sequences of at most `max_ctx` tokens (the kernel splits each
    actual context into that many equal parts itself).  Few, long-lived
    workgroups stream HBM best (profiles/r1_decode_parts.json: balanced parts
    6.0-6.4 TB/s vs 5.0-5.8 with fixed 512-token parts; target workgroup
    count re-swept in round 5, profiles/r5_decode_wgs_sweep.txt); small
    batches get more parts so the grid still covers the 256 CUs."""
    want = -(-DECODE_TARGET_WGS // max(1, batch * n_kv_heads))
    cap = -(-max(1, max_ctx) // DECODE_MIN_PART)
    return max(1, min(want, cap))


def decode_workspace(batch: int, n_q_heads: int, head_dim: int, n_parts: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    tmp_out = torch.empty((max(batch, 1), n_q_heads, n_parts, head_dim), dtype=torch.float32, device=device)
    tmp_ml = torch.empty((max(batch, 1), n_q_heads, n_parts, 2), dtype=torch.float32, device=device)
    return tmp_out, tmp_ml


def decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale, out, n_parts, workspace=None,
                     kv_scales=(1.0, 1.0)):
    """q: [B, Hq, D] (token stride q.stride(0)); out: [B, Hq, D] contiguous.
    n_parts: balanced partitions per sequence (decode_num_parts); workspace
    [B, Hq, n_parts, D] / [B, Hq, n_parts, 2] f32 when n_parts > 1.  An fp8
    cache is dequantized on load (K scale folded into the softmax scale)."""
    if not q.is_cuda:
        B = q.shape[0]
        cu = torch.arange(B + 1, dtype=torch.int32)
        out.copy_(ref.paged_attention(q, k_cache, v_cache, block_tables, cu, ctx_lens, scale, k_cache.shape[2],
                                      kv_scales))
        return out
    B, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    assert q.stride(1) == D and q.stride(2) == 1 and out.is_contiguous()
    assert block_tables.dtype == torch.int32 and ctx_lens.dtype == torch.int32
    if n_parts > 1:
        if workspace is None:
            workspace = decode_workspace(B, Hq, D, n_parts, q.device)
        tmp_out, tmp_ml = workspace
        assert tmp_out.shape[0] >= B and tmp_out.shape[2] == n_parts and tmp_ml.shape[2] == n_parts
        t0, t1 = tmp_out.data_ptr(), tmp_ml.data_ptr()
    else:
        t0 = t1 = 0
    _k().decode_attention(out.data_ptr(), t0, t1, q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                          block_tables.data_ptr(), block_tables.stride(0), ctx_lens.data_ptr(), B, Hq, Hkv, D, BS,
                          int(n_parts), float(scale), int(_kv_fp8(k_cache)), float(kv_scales[0]), float(kv_scales[1]),
                          _stream())
    return out


# the prefill-attention kernel: 8 waves (4 heads x 64 tokens share each K/V
# tile), LDS-DMA staging (the variants it beat: profiles/r1_prefill_attn_*.json)
PREFILL_WAVES = 91


def prefill_tile_tokens(n_q_heads: int, n_kv_heads: int) -> int:
    g = n_q_heads // n_kv_heads
    hpw = 4 if g >= 4 else g
    return (8 // hpw) * 32


def prefill_work_list(q_lens: list[int], ctx_lens: list[int], n_q_heads: int, n_kv_heads: int) -> list[int]:
    """Flattened (seq, first_token) pairs for the prefill kernel, heaviest first."""
    tt = prefill_tile_tokens(n_q_heads, n_kv_heads)
    items = []
    for s, (ql, cl) in enumerate(zip(q_lens, ctx_lens)):
        for t0 in range(0, ql, tt):
            cost = cl - ql + min(t0 + tt, ql)  # kv extent of the tile
            items.append((cost, s, t0))
    items.sort(key=lambda x: -x[0])
    flat = []
    for _, s, t0 in items:
        flat += [s, t0]
    return flat


# (device, stream) -> (K scratch, V scratch, arange) of the fp8 prefill path:
# one buffer per stream, sliced per call (block counts vary per step)
_KV_SCRATCH: dict = {}


def fp8_scratch_plan(ctx_lens: list[int], block_size: int, width: int, cap_blocks: int) -> list[tuple]:
    """Host side of the bounded fp8 prefill scratch: split the prefill
    sequences into consecutive groups whose live context blocks
    (ceil(ctx / block_size) each) fit `cap_blocks`, and pack each group's
    blocks densely.  Returns [(s0, s1, n_blocks, table)] with table an int32
    [s1 - s0, width] array: scratch block of (sequence, block).  A sequence
    alone never exceeds the cap (the runner sizes it >= max_model_len /
    block_size)."""
    import numpy as np

    nb = [-(-c // block_size) for c in ctx_lens]
    groups, s0 = [], 0
    while s0 < len(nb):
        s1, tot = s0, 0
        while s1 < len(nb) and (s1 == s0 or tot + nb[s1] <= cap_blocks):
            tot += nb[s1]
            s1 += 1
        tab = np.zeros((s1 - s0, width), dtype=np.int32)
        base = 0
        for i in range(s0, s1):
            tab[i - s0, :nb[i]] = np.arange(base, base + nb[i], dtype=np.int32)
            base += nb[i]
        groups.append((s0, s1, tot, tab))
        s0 = s1
    return groups


def kv_dequant_scratch(k_cache, v_cache, block_tables, ctx_lens, kv_scales=(1.0, 1.0), scratch=None):
    """fp8 cache -> bf16 copies of the prefill sequences' context blocks
    (csrc/kernels/rope_cache.hip kv_dequant): returns (K, V, block table) for
    the prefill attention kernel, which then reads bf16 tiles unchanged.
    `scratch` = (device int32 table [nseq, max_blocks], n_blocks) from
    :func:`fp8_scratch_plan` (the model runner's packed, capped layout:
    sum of ceil(ctx / block_size) blocks -- ADVICE r3: never
    nseq x padded max_blocks); without it (direct calls in tests) the
    dense table i * max_blocks + j."""
    nseq, maxb = block_tables.shape
    _, H, BS, D = k_cache.shape
    n = scratch[1] if scratch is not None else nseq * maxb
    key = (k_cache.device, _stream())
    ws = _KV_SCRATCH.get(key)
    if ws is None or ws[0].shape[0] < n or ws[0].shape[1:] != (H, BS, D):
        cap = max(n, 64)
        ws = (torch.empty((cap, H, BS, D), dtype=torch.bfloat16, device=k_cache.device),
              torch.empty((cap, H, BS, D), dtype=torch.bfloat16, device=k_cache.device),
              torch.arange(cap, dtype=torch.int32, device=k_cache.device))
        _KV_SCRATCH[key] = ws
    ks, vs = ws[0][:max(n, 1)], ws[1][:max(n, 1)]
    table = scratch[0] if scratch is not None else ws[2][:n].view(nseq, maxb)
    assert block_tables.dtype == torch.int32 and ctx_lens.dtype == torch.int32 and table.dtype == torch.int32
    assert table.shape == (nseq, maxb) and table.is_contiguous()
    _k().kv_dequant(k_cache.data_ptr(), v_cache.data_ptr(), ks.data_ptr(), vs.data_ptr(), block_tables.data_ptr(),
                    block_tables.stride(0), ctx_lens.data_ptr(), table.data_ptr(), nseq, maxb, H, BS, D,
                    float(kv_scales[0]), float(kv_scales[1]), _stream())
    return ks, vs, table


def prefill_attention(q, k_cache, v_cache, block_tables, cu_seqlens_q, ctx_lens, scale, out, work=None,
                      kv_scales=(1.0, 1.0), scratch=None, causal: bool = True):
    """q: [T, Hq, D] (token stride q.stride(0)); out: [T, Hq, D] contiguous.
    causal=False: every query attends to its sequence's whole context.

    `work` is the int32 device tensor from :func:`prefill_work_list`.  An fp8
    cache goes through :func:`kv_dequant_scratch` first (`scratch`: its packed
    table).
    """
    if not q.is_cuda:
        out.copy_(ref.paged_attention(q, k_cache, v_cache, block_tables, cu_seqlens_q, ctx_lens, scale, k_cache.shape[2],
                                      kv_scales, causal=causal))
        return out
    if _kv_fp8(k_cache):
        k_cache, v_cache, block_tables = kv_dequant_scratch(k_cache, v_cache, block_tables, ctx_lens, kv_scales,
                                                            scratch)
    T, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    assert q.stride(1) == D and q.stride(2) == 1 and out.is_contiguous()
    if work is None:
        cu = cu_seqlens_q.tolist()
        ql = [cu[i + 1] - cu[i] for i in range(len(cu) - 1)]
        work = torch.tensor(prefill_work_list(ql, ctx_lens.tolist(), Hq, Hkv), dtype=torch.int32, device=q.device)
    n_work = work.numel() // 2
    _k().prefill_attention(out.data_ptr(), q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                           block_tables.data_ptr(), block_tables.stride(0), cu_seqlens_q.data_ptr(),
                           ctx_lens.data_ptr(), work.data_ptr(), n_work, Hq, Hkv, D, BS, float(scale), int(causal),
                           PREFILL_WAVES, _stream())
    return out


def sample(logits, temperature=None, top_k=None, top_p=None, min_p=None, seeds=None, offsets=None,
           out_tokens=None, out_logprobs=None):
    """Returns (tokens int64 [B], logprobs f32 [B]).  All params are per-row tensors or None."""
    if not logits.is_cuda:
        t, lp = ref.sample(logits, temperature, top_k, top_p, min_p, seeds, offsets)
        if out_tokens is not None:
            out_tokens.copy_(t)
            out_logprobs.copy_(lp)
            return out_tokens, out_logprobs
        return t, lp
    B, V = logits.shape
    assert logits.stride(1) == 1
    dev = logits.device
    if out_tokens is None:
        out_tokens = torch.empty(B, dtype=torch.int64, device=dev)
    if out_logprobs is None:
        out_logprobs = torch.empty(B, dtype=torch.float32, device=dev)

    def p(t):
        return 0 if t is None else t.data_ptr()

    _k().sample(out_tokens.data_ptr(), out_logprobs.data_ptr(), logits.data_ptr(), int(logits.dtype == torch.float32),
                logits.stride(0), B, V, p(temperature), p(top_k), p(top_p), p(min_p), p(seeds), p(offsets), _stream())
    return out_tokens, out_logprobs


def sample_partial(logits, v0: int, temperature=None, seeds=None, offsets=None, out=None):
    """Per-rank half of vocab-parallel sampling (csrc/kernels/sampling.hip
    sample_partial_kernel): [B, 5] f32 rows {shard max, sum exp(x - max),
    race score of the shard winner, its global id, its logit}."""
    B, V = logits.shape
    if not logits.is_cuda:
        r = ref.sample_partial(logits, v0, temperature, seeds, offsets)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert logits.stride(1) == 1
    out = torch.empty((B, 5), dtype=torch.float32, device=logits.device) if out is None else out

    def p(t):
        return 0 if t is None else t.data_ptr()

    _k().sample_partial(out.data_ptr(), logits.data_ptr(), int(logits.dtype == torch.float32), logits.stride(0), B, V,
                        v0, p(temperature), p(seeds), p(offsets), _stream())
    return out


def combine_sampled_parts(parts: torch.Tensor, out_tokens=None, out_logprobs=None):
    """parts [W, B, 5] from every rank's sample_partial (rank order = vocab
    shard order) -> (tokens int64 [B], logprobs f32 [B]).  Device ops only
    (graph-capturable); identical on every rank."""
    m, s, score, idx, xb = parts.unbind(-1)
    M = m.max(0).values
    S = (s * torch.exp(m - M)).sum(0)
    w = score.argmax(0, keepdim=True)  # first maximum: the lowest shard wins ties
    tok = idx.gather(0, w).squeeze(0).to(torch.int64)
    lp = xb.gather(0, w).squeeze(0) - M - torch.log(S)
    if out_tokens is not None:
        out_tokens.copy_(tok)
        out_logprobs.copy_(lp)
        return out_tokens, out_logprobs
    return tok, lp


def apply_penalties(logits, output_tokens: list[list[int]], prompt_tokens: list[list[int]], rep, freq, pres):
    """In-place repetition/frequency/presence penalties (vLLM semantics)."""
    if not logits.is_cuda:
        return ref.apply_penalties(logits, output_tokens, prompt_tokens, rep, freq, pres)
    import numpy as np

    csr = [0]
    toks, counts, flags = [], [], []
    for outs, prompt in zip(output_tokens, prompt_tokens):
        cnt: dict[int, int] = {}
        for t in outs:
            cnt[t] = cnt.get(t, 0) + 1
        pset = set(prompt)
        for t in set(cnt) | pset:
            toks.append(t)
            counts.append(cnt.get(t, 0))
            flags.append((1 if t in cnt else 0) | (2 if t in pset else 0))
        csr.append(len(toks))
    dev = logits.device
    arr = lambda x, dt=np.int32: torch.from_numpy(np.asarray(x, dtype=dt)).to(dev, non_blocking=True)
    f32 = lambda x: torch.as_tensor(x, dtype=torch.float32).to(dev, non_blocking=True)
    tt = [arr(csr), arr(toks if toks else [0]), arr(counts if counts else [0]), arr(flags if flags else [0])]
    rr, ff, pp = f32(rep), f32(freq), f32(pres)
    _k().apply_penalties(logits.data_ptr(), int(logits.dtype == torch.float32), logits.stride(0), logits.shape[0],
                         tt[0].data_ptr(), tt[1].data_ptr(), tt[2].data_ptr(), tt[3].data_ptr(), rr.data_ptr(),
                         ff.data_ptr(), pp.data_ptr(), _stream())
    return logits


def kv_copy_blocks(dst: torch.Tensor, src: torch.Tensor, src_ids: torch.Tensor, dst_ids: torch.Tensor, n_prefix: int,
                   src_prefix_stride: int, dst_prefix_stride: int, src_block_bytes: int, dst_block_bytes: int,
                   copy_bytes: int, src_inner_off: int = 0, dst_inner_off: int = 0, stream: int | None = None,
                   dst_ptr: int | None = None, src_ptr: int | None = None):
    """Block gather/scatter over byte-addressed [prefix][block][inner] views.

    dst/src may be device tensors or pinned host tensors (pass their device-
    mapped pointers via dst_ptr/src_ptr for zero-copy host access).
    """
    on_gpu = src_ids.is_cuda
    if not on_gpu:
        return ref.kv_copy_blocks(dst, src, src_ids, dst_ids, n_prefix, src_prefix_stride, dst_prefix_stride,
                                  src_block_bytes, dst_block_bytes, src_inner_off, dst_inner_off, copy_bytes)
    assert src_ids.dtype == torch.int32 and dst_ids.dtype == torch.int32
    _k().kv_copy_blocks(dst.data_ptr() if dst_ptr is None else dst_ptr, src.data_ptr() if src_ptr is None else src_ptr,
                        src_ids.data_ptr(), dst_ids.data_ptr(), src_ids.numel(), n_prefix, src_prefix_stride,
                        dst_prefix_stride, src_block_bytes, dst_block_bytes, src_inner_off, dst_inner_off, copy_bytes,
                        _stream() if stream is None else stream)


def softmax_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)
