"""Plain-PyTorch fp32 reference implementations of every engine op.

They serve two purposes: (1) the numerics oracle for the HIP kernel tests
(``tests/test_kernels_gpu.py``) and (2) the execution path for CPU tensors so
the whole engine (scheduler, paged KV, prefix cache, disaggregation) can be
exercised in CPU-only CI with a tiny model.  They are never used for GPU
tensors -- see :mod:`dynamo_exp_amd.ops`.
"""
from __future__ import annotations

import math

import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * w.float()).to(x.dtype)


def add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """residual <- residual + x (in place); returns rmsnorm(residual) * w."""
    residual.copy_((residual.float() + x.float()).to(residual.dtype))
    return rmsnorm(residual, w, eps)


FP8_MAX = 448.0  # largest normal of OCP e4m3fn (gfx950's fp8)


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x @ w.T with fp32 accumulation, rounded to x's dtype."""
    return (x.float() @ w.float().t()).to(x.dtype)


def quant_fp8_rows(y: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Dynamic per-row e4m3fn quantisation: y ~= q * s, s = max|y_row| / 448."""
    yf = y.float()
    s = (yf.abs().amax(dim=-1, keepdim=True).clamp(min=1e-6) / FP8_MAX)
    q = (yf / s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q, s


def quant_fp8_weight(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-output-channel e4m3fn weight quantisation: w [N, K] ~= q * s[N]."""
    wf = w.float()
    s = wf.abs().amax(dim=1).clamp(min=1e-8) / FP8_MAX
    q = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q, s


def fp8_linear(x8: torch.Tensor, sx: torch.Tensor, w8: torch.Tensor, sw: torch.Tensor, out_dtype=torch.bfloat16):
    """(x8 * sx) @ (w8 * sw).T in fp32 -> out_dtype."""
    return ((x8.float() * sx.float()) @ (w8.float() * sw.float().view(-1, 1)).t()).to(out_dtype)


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: dict | None = None) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: cos in [:, :D/2], sin in [:, D/2:].

    Supports the llama3 frequency scaling (rope_type == "llama3") and linear.
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        rtype = scaling.get("rope_type", scaling.get("type"))
        if rtype == "llama3":
            factor = scaling["factor"]
            lf = scaling.get("low_freq_factor", 1.0)
            hf = scaling.get("high_freq_factor", 4.0)
            old = scaling.get("original_max_position_embeddings", 8192)
            low_wl, high_wl = old / lf, old / hf
            wl = 2 * math.pi / inv
            smooth = (old / wl - lf) / (hf - lf)
            scaled = torch.where(wl > low_wl, inv / factor, inv)
            mid = (wl <= low_wl) & (wl >= high_wl)
            inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        elif rtype == "linear":
            inv = inv / scaling["factor"]
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float()


def apply_rope(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x: [T, H, D] -> rotated (neox/rotate-half form), fp32 math."""
    d = x.shape[-1]
    cs = cos_sin[pos.long()]
    c, s = cs[:, None, : d // 2], cs[:, None, d // 2 :]
    x1, x2 = x[..., : d // 2].float(), x[..., d // 2 :].float()
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


def rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, n_q, n_kv, head_dim, block_size, rotate_q=True,
               kv_scales=(1.0, 1.0)):
    T = qkv.shape[0]
    q = qkv[:, : n_q * head_dim].view(T, n_q, head_dim)
    k = qkv[:, n_q * head_dim : (n_q + n_kv) * head_dim].view(T, n_kv, head_dim)
    v = qkv[:, (n_q + n_kv) * head_dim : (n_q + 2 * n_kv) * head_dim].view(T, n_kv, head_dim)
    if rotate_q:
        q.copy_(apply_rope(q, positions, cos_sin))
    k.copy_(apply_rope(k, positions, cos_sin))
    if slot_mapping is not None:
        write_kv(k, v, slot_mapping, k_cache, v_cache, block_size, kv_scales)


FP8_MAX = 448.0


def to_cache(x, cache_dtype, scale: float = 1.0):
    """Values as the KV cache stores them: bf16, or e4m3fn of x / scale clamped
    to +-448 (the kernels' v_cvt_pk_fp8_f32 after a clamp)."""
    if cache_dtype == torch.float8_e4m3fn:
        return (x.float() / scale).clamp(-FP8_MAX, FP8_MAX).to(cache_dtype)
    return x.to(cache_dtype)


def write_kv(k, v, slot_mapping, k_cache, v_cache, block_size, kv_scales=(1.0, 1.0)):
    """k, v: [T, Hkv, D]; caches [NB, Hkv, BS, D] (bf16 or fp8 e4m3fn with per-tensor scales)."""
    sm = slot_mapping.long()
    ok = sm >= 0
    if not bool(ok.any()):
        return
    sm, kk, vv = sm[ok], k[ok], v[ok]
    blk, off = sm // block_size, sm % block_size
    k_cache[blk, :, off] = to_cache(kk, k_cache.dtype, kv_scales[0])
    v_cache[blk, :, off] = to_cache(vv, v_cache.dtype, kv_scales[1])


def interleave_gate_up(w: torch.Tensor, blk: int = 32) -> torch.Tensor:
    """[gate; up] rows ([2F, K]) -> rows interleaved in blocks of `blk`:
    g[0:blk], u[0:blk], g[blk:2blk], u[blk:2blk], ... (the fused SwiGLU
    GEMM's weight layout, csrc/kernels/gemm256.hip)."""
    f2, k = w.shape
    f = f2 // 2
    g, u = w[:f].reshape(f // blk, blk, k), w[f:].reshape(f // blk, blk, k)
    return torch.stack([g, u], dim=1).reshape(f2, k)


def deinterleave_gate_up(w: torch.Tensor, blk: int = 32) -> torch.Tensor:
    f2, k = w.shape
    v = w.reshape(f2 // (2 * blk), 2, blk, k)
    return torch.cat([v[:, 0].reshape(-1, k), v[:, 1].reshape(-1, k)], 0)


def silu_and_mul(gate_up: torch.Tensor, blk: int = 0) -> torch.Tensor:
    """SwiGLU of [gate | up] columns (blk = 0) or of columns interleaved in
    blocks of `blk` (gate block, up block, ...)."""
    f = gate_up.shape[-1] // 2
    if blk:
        v = gate_up.reshape(*gate_up.shape[:-1], f // blk, 2, blk)
        g, u = v[..., 0, :].reshape(*gate_up.shape[:-1], f).float(), v[..., 1, :].reshape(*gate_up.shape[:-1], f).float()
    else:
        g, u = gate_up[..., :f].float(), gate_up[..., f:].float()
    return (torch.nn.functional.silu(g) * u).to(gate_up.dtype)


def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return table[ids.long()]


def _gather_kv(cache, block_table_row, n_tokens, block_size):
    nb = (n_tokens + block_size - 1) // block_size
    blocks = block_table_row[:nb].long()
    kv = cache[blocks]  # [nb, Hkv, BS, D]
    kv = kv.permute(0, 2, 1, 3).reshape(nb * block_size, cache.shape[1], cache.shape[3])
    return kv[:n_tokens]


def paged_attention(q, k_cache, v_cache, block_tables, cu_seqlens_q, ctx_lens, scale, block_size, kv_scales=(1.0, 1.0),
                    causal: bool = True):
    """Causal attention of new tokens over their paged context (prefix + new);
    causal=False: every query sees the whole context.

    q: [T, Hq, D]; returns [T, Hq, D].  Decode is the special case qlen == 1.
    """
    T, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    out = torch.empty_like(q)
    cu = cu_seqlens_q.tolist()
    cl = ctx_lens.tolist()
    for b in range(len(cl)):
        s, e, ctx = cu[b], cu[b + 1], cl[b]
        ql = e - s
        if ql == 0:
            continue
        k = _gather_kv(k_cache, block_tables[b], ctx, block_size).float() * kv_scales[0]  # [ctx, Hkv, D]
        v = _gather_kv(v_cache, block_tables[b], ctx, block_size).float() * kv_scales[1]
        k = k.repeat_interleave(G, dim=1)
        v = v.repeat_interleave(G, dim=1)
        qq = q[s:e].float()
        scores = torch.einsum("qhd,khd->hqk", qq, k) * scale
        qpos = torch.arange(ctx - ql, ctx, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        if causal:
            mask = kpos[None, :] > qpos[:, None]
            scores.masked_fill_(mask[None], float("-inf"))
        p = torch.softmax(scores, dim=-1)
        out[s:e] = torch.einsum("hqk,khd->qhd", p, v).to(q.dtype)
    return out


def sample(logits, temperature, top_k, top_p, min_p, seeds=None, offsets=None):
    """Reference sampler: greedy when T == 0, else filtered multinomial.

    Not bit-identical to the kernel's exponential race (different RNG); used
    for CPU execution and distributional tests.
    """
    lf = logits.float()
    B, V = lf.shape
    logp = torch.log_softmax(lf, dim=-1)
    out = torch.empty(B, dtype=torch.long)
    for i in range(B):
        t = float(temperature[i]) if temperature is not None else 0.0
        if t <= 0:
            out[i] = int(torch.argmax(lf[i]))
            continue
        x = lf[i] / t
        keep = torch.ones(V, dtype=torch.bool)
        k = int(top_k[i]) if top_k is not None else 0
        if 0 < k < V:
            kth = torch.topk(lf[i], k).values[-1]
            keep &= lf[i] >= kth
        mp = float(min_p[i]) if min_p is not None else 0.0
        if mp > 0:
            keep &= lf[i] >= lf[i].max() + t * math.log(mp)
        p = float(top_p[i]) if top_p is not None else 1.0
        if p < 1.0:
            probs = torch.softmax(x.masked_fill(~keep, float("-inf")), -1)
            sp, idx = torch.sort(probs, descending=True)
            cum = torch.cumsum(sp, 0)
            n = int((cum < p).sum()) + 1
            thr = sp[n - 1]
            keep &= probs >= thr
        probs = torch.softmax(x.masked_fill(~keep, float("-inf")), -1)
        g = None
        if seeds is not None:
            g = torch.Generator().manual_seed(int(seeds[i]) * 1000003 + int(offsets[i]) if offsets is not None else int(seeds[i]))
        out[i] = int(torch.multinomial(probs, 1, generator=g))
    lp = logp.gather(1, out[:, None]).squeeze(1)
    return out, lp


_M64 = (1 << 64) - 1


def _i64(c: int) -> int:
    return c - (1 << 64) if c >= 1 << 63 else c


def _srl(z: torch.Tensor, k: int) -> torch.Tensor:
    return (z >> k) & ((1 << (64 - k)) - 1)  # logical shift on int64


def _mix64(z: torch.Tensor) -> torch.Tensor:
    z = z + _i64(0x9E3779B97F4A7C15)
    z = (z ^ _srl(z, 30)) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(z, 27)) * _i64(0x94D049BB133111EB)
    return z ^ _srl(z, 31)


def uniform_hash(seed: int, offset: int, ids: torch.Tensor) -> torch.Tensor:
    """The sampling kernels' counter-based uniform in (0, 1) (sampling.hip
    `uniform`), in int64 torch arithmetic (wrapping multiply = mod 2^64)."""
    seed = torch.tensor(_i64(seed & _M64), dtype=torch.int64)
    inner = _mix64(torch.tensor(_i64((offset * 0xD1B54A32D192ED03) & _M64), dtype=torch.int64) + ids.to(torch.int64))
    h = _mix64(seed ^ inner)
    return (_srl(h, 40).to(torch.float64) + 0.5) * (1.0 / 16777216.0)


def sample_partial(logits, v0: int, temperature=None, seeds=None, offsets=None) -> torch.Tensor:
    lf = logits.float()
    B, V = lf.shape
    out = torch.empty(B, 5)
    ids = torch.arange(v0, v0 + V)
    for i in range(B):
        x = lf[i]
        m = x.max()
        t = float(temperature[i]) if temperature is not None else 0.0
        if t > 0:
            u = uniform_hash(int(seeds[i]) if seeds is not None else 0, int(offsets[i]) if offsets is not None else 0,
                             ids)
            score = (x.double() / t - torch.log(-torch.log(u))).float()
        else:
            score = x
        b = int(torch.argmax(score))
        out[i] = torch.tensor([m, torch.exp(x - m).sum(), score[b], v0 + b, x[b]])
    return out


def apply_penalties(logits, output_tokens: list, prompt_tokens: list, rep, freq, pres):
    for i in range(logits.shape[0]):
        row = logits[i]
        r, f, p = float(rep[i]), float(freq[i]), float(pres[i])
        outs = output_tokens[i]
        seen = set(outs) | set(prompt_tokens[i])
        if r != 1.0:
            for t in seen:
                v = row[t]
                row[t] = v / r if v > 0 else v * r
        if f or p:
            cnt = {}
            for t in outs:
                cnt[t] = cnt.get(t, 0) + 1
            for t, c in cnt.items():
                row[t] = row[t] - f * c - p
    return logits


def kv_copy_blocks(dst: torch.Tensor, src: torch.Tensor, src_ids, dst_ids, n_prefix, src_prefix_stride, dst_prefix_stride,
                   src_block_bytes, dst_block_bytes, src_inner_off, dst_inner_off, copy_bytes):
    d = dst.view(torch.uint8).reshape(-1)
    s = src.view(torch.uint8).reshape(-1)
    for p in range(n_prefix):
        for si, di in zip(list(map(int, src_ids)), list(map(int, dst_ids))):
            so = p * src_prefix_stride + si * src_block_bytes + src_inner_off
            do = p * dst_prefix_stride + di * dst_block_bytes + dst_inner_off
            d[do : do + copy_bytes] = s[so : so + copy_bytes]
