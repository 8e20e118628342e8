"""First-party Llama-family model for the MI355X engine.

Forward pass per layer (T tokens, all bf16; one fused op per line):
    x   = add_rmsnorm(h, residual)          HIP  (residual stream kept in place)
    qkv = x @ Wqkv^T                        hipBLASLt (fused Q|K|V projection)
    rope_cache(qkv -> q rot, K/V -> cache)  HIP  (rotary + paged-KV write fused)
    a   = paged attention(q, cache)         HIP  (prefill: MFMA flash; decode: split-K)
    h   = a @ Wo^T  [+ TP all-reduce]       hipBLASLt + RCCL / one-shot xGMI AR
    x   = add_rmsnorm(h, residual)          HIP
    a   = silu(x @ Wg^T) * (x @ Wu^T)       HIP MFMA GEMM with the SwiGLU epilogue
                                            (prefill; decode: GEMM + silu_and_mul)
    h   = a @ Wd^T [+ AR]                   hipBLASLt

Tensor parallelism is Megatron style (column-parallel QKV / gate-up, row-
parallel O / down, vocab-parallel LM head), one process per GPU.  The
reference delegates all of this to vLLM (`lib/engines/vllm0_8/src/lib.rs:371`);
see SURVEY.md §2.15 for the kernel inventory.
"""
from __future__ import annotations

import glob
import math
import os
from dataclasses import dataclass

import torch

from .. import ops
from ..ops import reference as ref
from ..utils import streams
from .config import ModelConfig


@dataclass
class AttnMeta:
    """Per-step attention metadata (device tensors)."""

    is_prefill: bool
    positions: torch.Tensor  # [T] int32/int64
    slot_mapping: torch.Tensor  # [T] int64 (-1 = do not write)
    block_tables: torch.Tensor  # [B, max_blocks] int32
    ctx_lens: torch.Tensor  # [B] int32 (tokens in cache incl. this step)
    logits_idx: torch.Tensor | None = None  # [B] rows of the hidden states that produce logits
    # prefill only
    cu_seqlens_q: torch.Tensor | None = None  # [B+1] int32
    work: torch.Tensor | None = None  # prefill kernel work list
    # decode only
    n_parts: int = 1  # balanced decode-attention partitions (ops.decode_num_parts)
    workspace: tuple | None = None
    # mixed steps: the first num_prefill_tokens rows are prompt chunks, the
    # remaining rows decode tokens described by `decode`
    num_prefill_tokens: int = 0
    decode: "AttnMeta | None" = None
    # fp8 KV cache, prefill rows: the packed bf16 dequant scratch
    # (ops.fp8_scratch_plan): one group -> fp8_scratch = (device table,
    # n_blocks); several (their blocks exceed the runner's cap) ->
    # fp8_groups = [(t0, t1, s0, s1, cu, work, table, n_blocks)], attention per group
    fp8_scratch: tuple | None = None
    fp8_groups: list | None = None
    # multimodal: rows of the token stream whose embeddings are replaced
    mm_rows: torch.Tensor | None = None
    mm_embeds: torch.Tensor | None = None


class TPGroup:
    """Tensor-parallel communicator (RCCL via torch.distributed) plus an
    optional custom one-shot all-reduce over xGMI for small messages."""

    def __init__(self, group=None, rank: int = 0, size: int = 1, custom_ar=None):
        self.group, self.rank, self.size = group, rank, size
        self.custom_ar = custom_ar

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        if self.custom_ar is not None and self.custom_ar.should_use(x):
            return self.custom_ar.all_reduce(x)
        import torch.distributed as dist

        dist.all_reduce(x, group=self.group)
        return x

    def rowparallel_mm(self, x: torch.Tensor, w: torch.Tensor, mm) -> torch.Tensor:
        """all_reduce(x @ w.T) for a row-parallel projection (O, down): with
        the custom all-reduce the GEMM writes straight into the registered
        (IPC-shared) buffer, so no copy sits between the GEMM and the reduce."""
        if self.size == 1:
            return mm(x, w)
        ar = self.custom_ar
        shape = (x.shape[0], w.shape[0])
        if ar is not None and x.dtype == torch.bfloat16 and ar.fits(shape):
            buf = ar.buffer(shape)
            mm(x, w, out=buf)
            return ar.all_reduce(buf)
        return self.all_reduce(mm(x, w))

    def check(self) -> None:
        """Fail loudly if a custom all-reduce barrier timed out (its results
        are invalid); called by the TP driver after every engine step."""
        if self.custom_ar is not None:
            self.custom_ar.check()

    def _custom_gather(self, x: torch.Tensor) -> bool:
        return self.custom_ar is not None and x.is_cuda and self.custom_ar.fits_gather(x.contiguous())

    def _no_host_collective_in_capture(self, what: str) -> None:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"TP {what} inside a hipGraph capture needs the custom all-gather or RCCL; "
                               "this group would stage it through host memory")

    def gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        """[B, k] on every rank -> [world, B, k] (rank order)."""
        if self.size == 1:
            return x[None]
        import torch.distributed as dist

        if self._custom_gather(x):  # xGMI peer reads, graph-capturable
            return self.custom_ar.all_gather(x.contiguous())
        if x.is_cuda and self._device_collectives():
            return self._gather_rows_device(x)
        self._no_host_collective_in_capture("gather_rows")
        xc = x.detach().cpu().contiguous()  # gloo: gathers through host memory
        out = torch.empty((self.size,) + tuple(x.shape), dtype=x.dtype)
        dist.all_gather(list(out.unbind(0)), xc, group=self.group)
        return out.to(x.device)

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        import torch.distributed as dist

        if self._custom_gather(x):  # [world, B, n] -> [B, world * n]
            g = self.custom_ar.all_gather(x.contiguous())
            return g.movedim(0, -2).reshape(*x.shape[:-1], self.size * x.shape[-1])
        if x.is_cuda and self._device_collectives():
            return self._all_gather_last_device(x)
        if x.is_cuda:
            self._no_host_collective_in_capture("all_gather_last")
        xc = x.detach().cpu().contiguous() if x.is_cuda else x.contiguous()
        parts = [torch.empty_like(xc) for _ in range(self.size)]
        dist.all_gather(parts, xc, group=self.group)
        return torch.cat(parts, dim=-1).to(x.device)

    # the device-collective (RCCL) forms: one all_gather_into_tensor into a
    # [world, ...] buffer on the tensor's own device (graph-capturable with
    # RCCL); tests/test_tp.py runs them over gloo on CPU tensors
    def _gather_rows_device(self, x: torch.Tensor) -> torch.Tensor:
        import torch.distributed as dist

        # rank-major flat output ([world * B, ...]: the shape gloo requires,
        # the same bytes RCCL writes), viewed as [world, B, ...]
        out = torch.empty((self.size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
        return out.view((self.size,) + tuple(x.shape))

    def _all_gather_last_device(self, x: torch.Tensor) -> torch.Tensor:
        g = self._gather_rows_device(x)  # [world, *, n] -> [*, world * n]
        return g.movedim(0, -2).reshape(*x.shape[:-1], self.size * x.shape[-1])

    def _device_collectives(self) -> bool:
        """True when the group's backend moves device tensors itself (RCCL);
        a gloo group on GPU tensors (several TP ranks sharing one GPU in
        tests) stages gathers through host memory."""
        import torch.distributed as dist

        return dist.get_backend(self.group) == "nccl"


class LlamaForCausalLM:
    def __init__(self, cfg: ModelConfig, device: torch.device | str = "cuda", dtype=torch.bfloat16,
                 tp: TPGroup | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPGroup()
        # mixed steps: run the (memory-bound) decode attention on a side stream
        # concurrently with the (MFMA-bound) prefill attention of the same layer
        self.overlap_decode_attn = os.environ.get("DX_OVERLAP_DECODE_ATTN", "0") != "0"
        self._side = None
        ts = self.tp.size
        if cfg.num_attention_heads % ts or cfg.intermediate_size % ts or cfg.vocab_size % ts:
            raise ValueError(f"model dims not divisible by tp={ts}")
        self.n_q = cfg.num_attention_heads // ts
        if cfg.num_key_value_heads >= ts:
            if cfg.num_key_value_heads % ts:
                raise ValueError("kv heads not divisible by tp")
            self.n_kv = cfg.num_key_value_heads // ts
        else:  # replicate kv heads across ranks
            self.n_kv = 1
        self.head_dim = cfg.head_dim
        if self.device.type == "cuda":
            # the gfx950 attention kernels (attn_prefill.hip, attn_decode.hip) are
            # built for head_dim 128 and 1 / 2 / 4 / 8 / 16 query heads per KV head:
            # refuse other shapes here rather than at the first forward
            g = self.n_q // self.n_kv
            if cfg.head_dim != 128 or self.n_q % self.n_kv or g not in (1, 2, 4, 8, 16):
                raise ValueError(f"unsupported attention shape on the GPU: head_dim {cfg.head_dim}, {self.n_q} query "
                                 f"/ {self.n_kv} KV heads per rank (kernels: head_dim 128, 1-16 query heads per KV "
                                 f"head in powers of two)")
        self.ffn = cfg.intermediate_size // ts
        self.vocab_local = cfg.vocab_size // ts
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.layers: list[dict[str, torch.Tensor]] = []
        self.embed = None
        self.norm = None
        self.lm_head = None
        self.cos_sin = ref.rope_cos_sin(cfg.head_dim, cfg.max_position_embeddings, cfg.rope_theta,
                                        cfg.rope_scaling).to(self.device)
        self.fp8 = False  # w8a8 e4m3fn linears (quantize_fp8)
        # per-tensor K / V scales of an fp8 KV cache (kv_cache_dtype="fp8"):
        # stored value = x / scale; 1.0 = uncalibrated, as vLLM's default
        self.kv_scales = (1.0, 1.0)
        self.kv_amax: torch.Tensor | None = None  # [2] running max |K|, |V| while calibrating
        # (M, N, K) -> (bn, bm, splits) of the small-M MFMA GEMM, filled by
        # tune_gemms() for the decode batch sizes; other shapes use hipBLASLt
        self.gemm_plan: dict[tuple[int, int, int], tuple] = {}
        self.gemm_tuned: set[tuple[int, int, int]] = set()  # shapes already decided (kernel or library)
        # (ceil(M / 256), N, K) of prefill-size qkv / o / down GEMMs routed to
        # gemm256 instead of hipBLASLt (tune_prefill_gemms)
        self.prefill_plan: set[tuple[int, int, int]] = set()
        # gate_up rows interleaved in blocks of gu_blk (enable_fused_mlp): token
        # counts >= fused_mlp_min_m run the fused SwiGLU GEMM (csrc/kernels/gemm256.hip)
        self.gu_blk = 0
        # decode sizes whose gate_up runs the deep-stream kernel's SwiGLU form: (M, N, K) -> config
        self.gemm_plan_silu: dict[tuple[int, int, int], tuple] = {}
        # disagg prefill worker: called as layer_hook(i) once layer i's KV is in
        # the cache during prefill forwards (layer-streamed KV transfer)
        self.layer_hook = None
        self.fused_mlp_min_m = int(os.environ.get("DX_FUSED_MLP_MIN_M", "512"))
        # RMSNorm weights folded into the projections (fold_norms); forwards of
        # at least fold_min_m tokens run _forward_folded
        self.norm_folded = False
        self.fold_min_m = int(os.environ.get("DX_FOLD_MIN_M", "512"))

    # ------------------------------------------------------------------ weights
    def random_init(self, seed: int = 0) -> "LlamaForCausalLM":
        """Random weights of the real architecture (no checkpoints offline).

        Scaled so activations stay O(1) through all layers (std 1/sqrt(fan_in)
        for projections), i.e. realistic kernel inputs rather than zeros.
        """
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev).manual_seed(seed + 7919 * self.tp.rank)
        H = cfg.hidden_size

        def rnd(*shape, std):
            t = torch.empty(*shape, device=dev, dtype=dt)
            t.normal_(0.0, std, generator=g)
            return t

        qkv_rows = (self.n_q + 2 * self.n_kv) * self.head_dim
        self.layers = []
        for _ in range(cfg.num_hidden_layers):
            self.layers.append(
                dict(
                    ln1=torch.ones(H, device=dev, dtype=dt),
                    ln2=torch.ones(H, device=dev, dtype=dt),
                    qkv=rnd(qkv_rows, H, std=1 / math.sqrt(H)),
                    o=rnd(H, self.n_q * self.head_dim, std=1 / math.sqrt(cfg.q_size) / math.sqrt(cfg.num_hidden_layers)),
                    gate_up=rnd(2 * self.ffn, H, std=1 / math.sqrt(H)),
                    down=rnd(H, self.ffn, std=1 / math.sqrt(cfg.intermediate_size) / math.sqrt(cfg.num_hidden_layers)),
                )
            )
        self.embed = rnd(cfg.vocab_size, H, std=1.0)
        self.norm = torch.ones(H, device=dev, dtype=dt)
        self.lm_head = self.embed[self.tp.rank * self.vocab_local:(self.tp.rank + 1) * self.vocab_local] \
            if cfg.tie_word_embeddings else rnd(self.vocab_local, H, std=1 / math.sqrt(H))
        return self

    def load_safetensors(self, path: str) -> "LlamaForCausalLM":
        """Load HF Llama safetensors (sharded for this TP rank)."""
        from safetensors import safe_open

        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            raise FileNotFoundError(f"no safetensors in {path}")
        tensors = {}
        for f in files:
            with safe_open(f, framework="pt", device="cpu") as sf:
                for k in sf.keys():
                    tensors[k] = sf.get_tensor(k)
        cfg, r, ts = self.cfg, self.tp.rank, self.tp.size
        D = self.head_dim

        def shard_rows(t, n):
            return t.view(-1, t.shape[-1]) if ts == 1 else t.chunk(ts, dim=0)[r] if n is None else t

        def cast(t):
            return t.to(self.device, self.dtype).contiguous()

        def kv_shard(t):
            if cfg.num_key_value_heads >= ts:
                return t.view(cfg.num_key_value_heads, D, -1).chunk(ts, dim=0)[r].reshape(-1, t.shape[-1])
            return t.view(cfg.num_key_value_heads, D, -1)[r * cfg.num_key_value_heads // ts].reshape(-1, t.shape[-1])

        self.layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"model.layers.{i}."
            q = tensors[p + "self_attn.q_proj.weight"].chunk(ts, 0)[r]
            k = kv_shard(tensors[p + "self_attn.k_proj.weight"])
            v = kv_shard(tensors[p + "self_attn.v_proj.weight"])
            gate = tensors[p + "mlp.gate_proj.weight"].chunk(ts, 0)[r]
            up = tensors[p + "mlp.up_proj.weight"].chunk(ts, 0)[r]
            self.layers.append(dict(
                ln1=cast(tensors[p + "input_layernorm.weight"]),
                ln2=cast(tensors[p + "post_attention_layernorm.weight"]),
                qkv=cast(torch.cat([q, k, v], 0)),
                o=cast(tensors[p + "self_attn.o_proj.weight"].chunk(ts, 1)[r]),
                gate_up=cast(torch.cat([gate, up], 0)),
                down=cast(tensors[p + "mlp.down_proj.weight"].chunk(ts, 1)[r]),
            ))
        self.embed = cast(tensors["model.embed_tokens.weight"])
        self.norm = cast(tensors["model.norm.weight"])
        lm = tensors.get("lm_head.weight", tensors["model.embed_tokens.weight"])
        self.lm_head = cast(lm.chunk(ts, 0)[r])
        return self

    def load_shard_from(self, full: "LlamaForCausalLM") -> "LlamaForCausalLM":
        """Take this rank's TP shard of a full (tp=1) model's weights (tests)."""
        r, ts, D = self.tp.rank, self.tp.size, self.head_dim
        cfg = self.cfg
        q_sz, kv_sz = cfg.q_size, cfg.kv_size
        self.layers = []
        for L in full.layers:
            q, k, v = L["qkv"].split([q_sz, kv_sz, kv_sz], 0)

            def kvs(t):  # this rank's KV heads (one replicated head when TP > KV heads)
                h = t.view(cfg.num_key_value_heads, D, -1)
                if cfg.num_key_value_heads >= ts:
                    return h.chunk(ts, 0)[r].reshape(-1, t.shape[-1])
                return h[r * cfg.num_key_value_heads // ts].reshape(-1, t.shape[-1])

            F = cfg.intermediate_size
            g, u = L["gate_up"].split([F, F], 0)
            self.layers.append(dict(
                ln1=L["ln1"].to(self.device), ln2=L["ln2"].to(self.device),
                qkv=torch.cat([q.chunk(ts, 0)[r], kvs(k), kvs(v)], 0).contiguous().to(self.device),
                o=L["o"].chunk(ts, 1)[r].contiguous().to(self.device),
                gate_up=torch.cat([g.chunk(ts, 0)[r], u.chunk(ts, 0)[r]], 0).contiguous().to(self.device),
                down=L["down"].chunk(ts, 1)[r].contiguous().to(self.device)))
        self.embed = full.embed.to(self.device)
        self.norm = full.norm.to(self.device)
        self.lm_head = full.lm_head.chunk(ts, 0)[r].contiguous().to(self.device)
        return self

    LINEARS = ("qkv", "o", "gate_up", "down")

    def quantize_fp8(self) -> "LlamaForCausalLM":
        """w8a8 serving: every projection weight becomes e4m3fn with a per-output-
        channel fp32 scale; activations are quantised per token at run time by
        the kernels that produce them (ops.rmsnorm_quant / silu_mul_quant /
        quant_rows) and the GEMMs run on hipBLASLt's fp8 path.  Embedding, LM
        head, norms and the KV cache stay bf16.  The same recipe as FP8
        checkpoints served by the reference's vLLM workers (dynamic per-token
        activations, static per-channel weights)."""
        self.gemm_plan_silu.clear()
        if self.gu_blk:  # the fp8 path's silu_mul_quant takes [gate | up] halves
            for L in self.layers:
                L["gate_up"] = ref.deinterleave_gate_up(L["gate_up"], self.gu_blk).contiguous()
            self.gu_blk = 0
        for L in self.layers:
            for name in self.LINEARS:
                q, s = ref.quant_fp8_weight(L.pop(name))
                L[name + "_q"] = q.contiguous()
                L[name + "_s"] = s.view(1, -1).contiguous()
        self.fp8 = True
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        return self

    def enable_fused_mlp(self) -> bool:
        """Interleave every layer's gate_up rows in blocks of 32 (gate, up, gate,
        ...) so prefill-sized MLPs run the hand-written GEMM with the SwiGLU
        epilogue: the [T, 2F] gate/up intermediate is never materialised
        (profiles/r2_gemm256.txt: 1314-1336 vs 1374-1379 us for hipBLASLt + silu_and_mul
        at 8192 tokens).  Decode-sized batches keep the library / small-M GEMM
        and an interleave-aware silu_and_mul.  bf16 GPU models only."""
        if self.gu_blk or self.fp8 or self.device.type != "cuda" or not self.layers:
            return False
        if os.environ.get("DX_FUSED_MLP", "1") == "0":
            return False
        if (2 * self.ffn) % 256 or self.cfg.hidden_size % 128:
            return False
        blk = ops.GEMM256_BLK
        for L in self.layers:
            L["gate_up"] = ref.interleave_gate_up(L["gate_up"], blk).contiguous()
        self.gu_blk = blk
        torch.cuda.empty_cache()
        return True

    def mlp_act(self, x: torch.Tensor, L: dict) -> torch.Tensor:
        """silu(x @ Wg^T) * (x @ Wu^T) for the bf16 path: prefill sizes on the
        256x256 GEMM with the SwiGLU epilogue, decode sizes on the deep-stream
        kernel's SwiGLU form where the tuner adopted it (gemm_plan_silu), else
        GEMM + interleave-aware silu_and_mul."""
        M = x.shape[0]
        if self.gu_blk and M >= self.fused_mlp_min_m and ops.gemm256_ok(x, L["gate_up"]):
            return ops.gemm256(x, L["gate_up"], ops.GEMM256_EPI_SILU)
        if self.gemm_plan_silu and M <= ops.SKINNY_MAX_M:
            w = L["gate_up"]
            cfg = self.gemm_plan_silu.get((M, w.shape[0], w.shape[1]))
            if cfg is not None and x.data_ptr() % 16 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0:
                return ops.dstream_linear(x, w, cfg, silu=True)
        return ops.silu_and_mul(self._mm(x, L["gate_up"]), blk=self.gu_blk)

    @torch.no_grad()
    def warmup_linears(self, tokens: int) -> None:
        """Run every projection GEMM of one layer at M = tokens so the GEMM
        library has selected (and loaded from disk) its kernels for this size
        before serving -- on a cold node the first use of a kernel family can
        stall a step for seconds."""
        L = self.layers[0]
        H = self.cfg.hidden_size
        x = torch.zeros(tokens, H, device=self.device, dtype=self.dtype)
        if self.fp8:
            x8, sx = ops.quant_rows(x)
            gu = ops.fp8_linear(x8, sx, L["gate_up_q"], L["gate_up_s"])
            ops.fp8_linear(x8, sx, L["qkv_q"], L["qkv_s"])
            a8, sa = ops.quant_rows(torch.zeros(tokens, self.n_q * self.head_dim, device=self.device, dtype=self.dtype))
            ops.fp8_linear(a8, sa, L["o_q"], L["o_s"])
            d8, sd = ops.silu_mul_quant(gu)
            ops.fp8_linear(d8, sd, L["down_q"], L["down_s"])
        else:
            torch.matmul(x, L["qkv"].t())
            torch.matmul(torch.zeros(tokens, self.n_q * self.head_dim, device=self.device, dtype=self.dtype),
                         L["o"].t())
            torch.matmul(self.mlp_act(x, L), L["down"].t())

    def weight_bytes(self) -> int:
        n = sum(t.numel() * t.element_size() for l in self.layers for t in l.values())
        n += self.embed.numel() * 2 + self.lm_head.numel() * 2
        return n

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches: list[tuple[torch.Tensor, torch.Tensor]]):
        """Returns final-normed hidden rows at meta.logits_idx (or all rows)."""
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        T = input_ids.shape[0]
        nq, nkv, D = self.n_q, self.n_kv, self.head_dim
        bs = kv_caches[0][0].shape[2]
        h = ops.embedding(input_ids, self.embed)
        if meta.mm_rows is not None:  # image features replace the placeholder tokens
            h.index_copy_(0, meta.mm_rows, meta.mm_embeds.to(h.dtype))
        if self._fold_ok(T):
            return self._forward_folded(h, meta, kv_caches, eps)
        residual = h
        x = None
        attn_out = torch.empty((T, nq, D), device=h.device, dtype=h.dtype)
        fp8 = self.fp8
        # single-GPU decode: the O / down projections may leave split-K partials
        # (ops.SplitK) that the following residual-add + RMSNorm sums itself;
        # the norm then writes into nbuf instead of in place
        mm_o = self._mm_partial if (self.tp.size == 1 and self.gemm_plan) else self._mm
        nbuf, qbuf = [], []

        def nout(t):
            if not isinstance(t, ops.SplitK):
                return t
            if not nbuf:
                nbuf.append(torch.empty((T, self.cfg.hidden_size), device=residual.device, dtype=residual.dtype))
            return nbuf[0]
        for i, L in enumerate(self.layers):
            if i == 0:
                residual = h.clone()
            if fp8:
                x8, sx = ops.rmsnorm_quant(h, residual if i else None, L["ln1"], eps)
                qkv = self._mm8(x8, sx, L, "qkv")
            else:
                x = ops.rmsnorm(h, L["ln1"], eps) if i == 0 else ops.add_rmsnorm(h, residual, L["ln1"], eps, out=nout(h))
                # the QKV partials (split-K plan) are summed by the rope kernel, which writes the whole row
                qkv = self._mm_partial(x, L["qkv"]) if self.gemm_plan else self._mm(x, L["qkv"])
            kc, vc = kv_caches[i]
            if isinstance(qkv, ops.SplitK):
                if not qbuf:
                    qbuf.append(torch.empty(qkv.shape, device=residual.device, dtype=residual.dtype))
                qkv = ops.rope_cache(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc, nq, nkv, D, bs,
                                     kv_scales=self.kv_scales, out=qbuf[0])
            else:
                ops.rope_cache(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc, nq, nkv, D, bs,
                               kv_scales=self.kv_scales)
            if self.layer_hook is not None and meta.is_prefill:
                self.layer_hook(i)
            if self.kv_amax is not None:  # fp8 KV-scale calibration (LLMEngine.calibrate_kv_scales)
                kv = qkv[:, nq * D:].view(T, 2, nkv * D).float().abs().amax(dim=(0, 2))
                self.kv_amax = torch.maximum(self.kv_amax, kv)
            self._attend(qkv[:, : nq * D].view(T, nq, D), kc, vc, meta, attn_out)
            if fp8:
                a8, sa = ops.quant_rows(attn_out.view(T, nq * D))
                h = self.tp.all_reduce(self._mm8(a8, sa, L, "o"))
                x8, sx = ops.rmsnorm_quant(h, residual, L["ln2"], eps)
                gu = self._mm8(x8, sx, L, "gate_up")
                a8, sa = ops.silu_mul_quant(gu)
                h = self.tp.all_reduce(self._mm8(a8, sa, L, "down"))
                continue
            h = self.tp.rowparallel_mm(attn_out.view(T, nq * D), L["o"], mm_o)
            x = ops.add_rmsnorm(h, residual, L["ln2"], eps, out=nout(h))
            a = self.mlp_act(x, L)
            h = self.tp.rowparallel_mm(a, L["down"], mm_o)
        if isinstance(h, ops.SplitK) and meta.logits_idx is not None:
            h = ops.splitk_reduce(h)
        if meta.logits_idx is not None:
            if meta.logits_idx.numel() == 0:
                return h[:0]
            h = h.index_select(0, meta.logits_idx)
            residual = residual.index_select(0, meta.logits_idx)
        return ops.add_rmsnorm(h, residual, self.norm, eps)

    def _attend(self, q: torch.Tensor, kc, vc, meta: AttnMeta, attn_out: torch.Tensor) -> None:
        """Paged attention of one layer: prefill rows on the prefill kernel,
        decode rows on the decode kernel (on the side stream beside it when
        overlap_decode_attn), into attn_out [T, nq, D]."""
        T = q.shape[0]
        if meta.is_prefill:
            Tp = meta.num_prefill_tokens if meta.decode is not None else T
            d = meta.decode
            side = self._side_stream() if (d is not None and Tp and q.is_cuda and self.overlap_decode_attn) else None
            if side is not None:  # fork point: the side stream may start once q and the KV writes are done
                side.wait_stream(torch.cuda.current_stream(q.device))
            if Tp and meta.fp8_groups:  # fp8 cache whose prefill context exceeds the scratch cap
                for t0, t1, s0, s1, cu_g, work_g, tab_g, nb_g in meta.fp8_groups:
                    ops.prefill_attention(q[t0:t1], kc, vc, meta.block_tables[s0:s1], cu_g, meta.ctx_lens[s0:s1],
                                          self.scale, attn_out[t0:t1], work=work_g, kv_scales=self.kv_scales,
                                          scratch=(tab_g, nb_g))
            elif Tp:
                # prefill attention first: one workgroup per CU (VGPR-bound, 2 waves/SIMD) leaves
                # room on every SIMD for one decode-attention wave streaming KV beside it
                ops.prefill_attention(q[:Tp], kc, vc, meta.block_tables, meta.cu_seqlens_q, meta.ctx_lens,
                                      self.scale, attn_out[:Tp], work=meta.work, kv_scales=self.kv_scales,
                                      scratch=meta.fp8_scratch)
            if side is not None:
                with torch.cuda.stream(side):
                    ops.decode_attention(q[Tp:], kc, vc, d.block_tables, d.ctx_lens, self.scale, attn_out[Tp:],
                                         d.n_parts, workspace=d.workspace, kv_scales=self.kv_scales)
            if side is not None:  # join before the O projection reads attn_out
                torch.cuda.current_stream(q.device).wait_stream(side)
            elif d is not None:
                ops.decode_attention(q[Tp:], kc, vc, d.block_tables, d.ctx_lens, self.scale, attn_out[Tp:],
                                     d.n_parts, workspace=d.workspace, kv_scales=self.kv_scales)
        else:
            ops.decode_attention(q, kc, vc, meta.block_tables, meta.ctx_lens, self.scale, attn_out,
                                 meta.n_parts, workspace=meta.workspace, kv_scales=self.kv_scales)

    # ------------------------------------------------------------------ folded norms
    def fold_norms(self) -> bool:
        """Fold the per-layer RMSNorm weights into the columns of the
        projections that consume the normed rows (qkv <- ln1, gate_up <- ln2):
        norm(h) @ W^T = (1 / rms(h)) * (h @ (W diag(w))^T).  The norms keep
        weight 1, so the unfused path computes the same model; large forwards
        (`_fold_ok`) then skip the norm kernels: the residual adds run as the
        o / down GEMMs' accumulation (beta = 1) and the row scale 1 / rms goes
        to the consumers (rope_cache for qkv, the fused SwiGLU GEMM's epilogue
        for gate_up).  bf16 projections only; idempotent."""
        if self.norm_folded or self.fp8 or os.environ.get("DX_FOLD_NORM", "1") == "0":
            return self.norm_folded
        for L in self.layers:
            for w_name, n_name in (("qkv", "ln1"), ("gate_up", "ln2")):
                w, g = L[w_name], L[n_name]
                L[w_name] = (w.float() * g.float()[None, :]).to(w.dtype).contiguous()
                L[n_name] = torch.ones_like(g)
        self.norm_folded = True
        return True

    def _fold_ok(self, T: int) -> bool:
        return (self.norm_folded and not self.fp8 and self.tp.size == 1 and self.kv_amax is None
                and T >= self.fold_min_m)

    def _forward_folded(self, h: torch.Tensor, meta: AttnMeta, kv_caches, eps: float) -> torch.Tensor:
        """forward() for large T on folded norms: per layer one row-rms read
        of the residual stream instead of two add + norm passes (read x and
        residual, write both), the residual adds inside the o / down GEMMs."""
        T = h.shape[0]
        nq, nkv, D = self.n_q, self.n_kv, self.head_dim
        bs = kv_caches[0][0].shape[2]
        res = h  # the embedding output: this forward's own buffer, accumulated in place
        attn_out = torch.empty((T, nq, D), device=h.device, dtype=h.dtype)
        rs = torch.empty(T, device=h.device, dtype=torch.float32)
        for i, L in enumerate(self.layers):
            ops.row_rrms(res, eps, out=rs)
            qkv = self._mm(res, L["qkv"])
            kc, vc = kv_caches[i]
            ops.rope_cache(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc, nq, nkv, D, bs,
                           kv_scales=self.kv_scales, row_scale=rs)
            if self.layer_hook is not None and meta.is_prefill:
                self.layer_hook(i)
            self._attend(qkv[:, : nq * D].view(T, nq, D), kc, vc, meta, attn_out)
            res.addmm_(attn_out.view(T, nq * D), L["o"].t())
            ops.row_rrms(res, eps, out=rs)
            if self.gu_blk and ops.gemm256_ok(res, L["gate_up"]):
                a = ops.gemm256(res, L["gate_up"], ops.GEMM256_EPI_SILU, row_scale=rs)
            else:
                gu = self._mm(res, L["gate_up"])
                a = ops.silu_and_mul((gu.float() * rs[:, None]).to(gu.dtype), blk=self.gu_blk)
            res.addmm_(a, L["down"].t())
        if meta.logits_idx is not None:
            if meta.logits_idx.numel() == 0:
                return res[:0]
            res = res.index_select(0, meta.logits_idx)
        return ops.rmsnorm(res, self.norm, eps)

    def _mm8(self, x8: torch.Tensor, sx: torch.Tensor, L: dict, name: str) -> torch.Tensor:
        """A w8a8 projection (hipBLASLt's fp8 GEMM)."""
        return ops.fp8_linear(x8, sx, L[name + "_q"], L[name + "_s"])

    def _mm_partial(self, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None):
        """_mm, but a split-K deep-stream plan returns its partials (ops.SplitK)."""
        return self._mm(x, w, out=out, partial=out is None)

    def _mm(self, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None, partial: bool = False):
        M = x.shape[0]
        if self.gemm_plan and M <= ops.SKINNY_MAX_M:
            cfg = self.gemm_plan.get((M, w.shape[0], w.shape[1]))
            if cfg is not None and x.data_ptr() % 16 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0:
                return ops.skinny_linear(x, w, cfg, out=out, partial=partial and os.environ.get("DX_SPLITK_FUSE", "1") != "0")
        elif self.prefill_plan and (-(-M // 256), w.shape[0], w.shape[1]) in self.prefill_plan and ops.gemm256_ok(x, w):
            return ops.gemm256(x, w, out=out)
        if out is not None:
            return torch.matmul(x, w.t(), out=out)
        return torch.matmul(x, w.t())

    @torch.no_grad()
    def tune_prefill_gemms(self, max_tokens: int, min_tokens: int = 2048, min_gain: float = 0.05,
                           reps: int = 2) -> list[dict]:
        """Per 256-token bucket of prefill-size M (min_tokens .. max_tokens)
        and plain projection (qkv / o / down), hipBLASLt vs the hand 256x256
        kernel (csrc/kernels/gemm256.hip, store epilogue), timed over this
        model's per-layer weights with random activations.  hipBLASLt's
        heuristic picks a slow kernel for some M (down at M 4353-4608,
        5377-5632, 6401-6656, 7425-7680: 1.4-1.6x slower than gemm256,
        profiles/r3_gemm_pad_probe.txt); those buckets are routed to gemm256."""
        if self.device.type != "cuda" or self.fp8 or not self.layers or os.environ.get("DX_PREFILL_TUNE", "1") == "0":
            return []
        groups = [[L[n] for L in self.layers] for n in ("qkv", "o", "down") if n in self.layers[0]]
        dev = self.device

        def timed(fn) -> float:
            fn()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(reps):
                fn()
            ev1.record()
            ev1.synchronize()
            return ev0.elapsed_time(ev1) * 1e3 / reps

        report = []
        for b in range(max(1, min_tokens // 256), -(-max_tokens // 256) + 1):
            M = 256 * b - 64  # inside the bucket (the library's choice depends on M, not the bucket edge)
            for ws in groups:
                N, K = ws[0].shape
                x = torch.randn(M, K, device=dev, dtype=self.dtype)
                if not ops.gemm256_ok(x, ws[0]):
                    continue
                sub = ws[:: max(1, len(ws) // 8)]  # 8 layers' weights: > the Infinity Cache, quick
                lib = timed(lambda: [torch.matmul(x, w.t()) for w in sub]) / len(sub)
                g = timed(lambda: [ops.gemm256(x, w) for w in sub]) / len(sub)
                adopt = g < lib * (1 - min_gain)
                if adopt:
                    self.prefill_plan.add((b, N, K))
                report.append({"bucket": b, "N": N, "K": K, "lib_us": round(lib, 1), "gemm256_us": round(g, 1),
                               "adopted": adopt})
        return report

    @torch.no_grad()
    def tune_gemms(self, sizes, min_gain: float = 0.03, reps: int = 2) -> list[dict]:
        """Pick, per decode batch size M <= 256 and projection shape, between
        hipBLASLt and the launch configurations of the hand-written small-M GEMMs
        (csrc/kernels/skinny_gemm.hip, dstream_gemm.hip), by timing each over this model's own
        per-layer weights in turn (their footprint exceeds the 256 MB Infinity
        Cache, so every call streams its weights from HBM as in a real step).
        A kernel config is adopted only when it beats the library by
        `min_gain`, after a numerics check against it.  Returns the timings."""
        if self.device.type != "cuda" or self.fp8 or not self.layers or os.environ.get("DX_SKINNY", "1") == "0":
            return []
        dev = self.device
        groups = [[L[n] for L in self.layers] for n in self.LINEARS] + [[self.lm_head]]
        # O / down partials are summed by the next norm (forward's mm_o), QKV's by
        # the rope kernel: time those projections without the reduction launch
        # they will not pay
        fuse_on = os.environ.get("DX_SPLITK_FUSE", "1") != "0"
        fused = {id(L[n]) for L in self.layers for n in (("qkv", "o", "down") if self.tp.size == 1 else ("qkv",))
                 if n in L} if fuse_on else set()

        def timed(fn) -> float:
            fn()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(reps):
                fn()
            ev1.record()
            ev1.synchronize()
            return ev0.elapsed_time(ev1) * 1e3 / reps

        report = []
        for M in sorted(set(int(m) for m in sizes)):
            if not 1 <= M <= ops.SKINNY_MAX_M:
                continue
            for ws in groups:
                N, K = ws[0].shape
                key = (M, N, K)
                if key in self.gemm_tuned:
                    continue
                self.gemm_tuned.add(key)
                x = torch.randn(M, K, device=dev, dtype=self.dtype)
                lib = timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws)
                best = None
                for cfg in ops.skinny_configs(M, N, K) + ops.dstream_tune_configs(M, N, K):
                    if cfg[0] != ops.DSTREAM and ((M <= 32 and cfg[1] == 64)
                                                                    or (cfg[0] == 128 and M <= 32)):
                        continue
                    part = id(ws[0]) in fused
                    t = timed(lambda: [ops.skinny_linear(x, w, cfg, partial=part) for w in ws]) / len(ws)
                    if best is None or t < best[0]:
                        best = (t, cfg)
                row = {"key": key, "lib_us": round(lib, 2), "best_us": None, "cfg": None, "adopted": False}
                if best is not None:
                    row["best_us"], row["cfg"] = round(best[0], 2), best[1]
                    if best[0] < lib * (1 - min_gain):
                        # numerics on the first and the last layer's weights (not layer 0 alone)
                        for w in (ws[0], ws[-1]):
                            want = torch.matmul(x, w.t()).float()
                            got = ops.skinny_linear(x, w, best[1]).float()
                            err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
                            if not err < 2e-2:
                                raise RuntimeError(f"skinny_gemm {best[1]} at {key}: relative error {err:.3g}")
                        self.gemm_plan[key] = best[1]
                        row["adopted"] = True
                if self.gu_blk == ops.GEMM256_BLK and ws[0] is self.layers[0].get("gate_up"):
                    self._tune_silu(key, x, ws, row, timed)
                report.append(row)
        return report

    def _tune_silu(self, key, x, ws, row, timed, min_gain: float = 0.01) -> None:
        """Decode gate_up: the deep-stream kernel's SwiGLU form (one launch,
        [M, F] output) against what the MLP runs otherwise -- the GEMM just
        picked (library or hand kernel) plus silu_and_mul.  Adopted into
        gemm_plan_silu when faster, after numerics on the first and last layer."""
        M = key[0]
        cur = self.gemm_plan.get(key)

        def current(w):
            g = ops.skinny_linear(x, w, cur) if cur is not None else torch.matmul(x, w.t())
            return ops.silu_and_mul(g, blk=self.gu_blk)

        base = timed(lambda: [current(w) for w in ws]) / len(ws)
        best = None
        for cfg in ops.dstream_tune_configs(*key):
            if cfg[2] != 2:
                continue
            t = timed(lambda: [ops.dstream_linear(x, w, cfg, silu=True) for w in ws]) / len(ws)
            if best is None or t < best[0]:
                best = (t, cfg)
        row["silu_base_us"] = round(base, 2)
        row["silu_best_us"], row["silu_cfg"] = (round(best[0], 2), best[1]) if best else (None, None)
        row["silu_adopted"] = False
        if best is None or not best[0] < base * (1 - min_gain):
            return
        for w in (ws[0], ws[-1]):
            want = current(w).float()
            got = ops.dstream_linear(x, w, best[1], silu=True).float()
            err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
            if not err < 2e-2:
                raise RuntimeError(f"dstream SwiGLU {best[1]} at {key}: relative error {err:.3g}")
        self.gemm_plan_silu[key] = best[1]
        row["silu_adopted"] = True

    def _side_stream(self):
        if self._side is None:
            self._side = streams.stream("side", self.device)  # high priority: utils/streams.py
        return self._side

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """Full-vocab logits (all-gathered over TP ranks)."""
        logits = self._mm(hidden, self.lm_head)
        return self.tp.all_gather_last(logits)

    def sample_sharded(self, hidden: torch.Tensor, temperature, seeds, offsets, out_tokens=None, out_logprobs=None):
        """Greedy / temperature sampling without gathering the logits: every
        rank runs the exponential race over its own vocab shard
        (ops.sample_partial) and the ranks exchange 5 floats per row (shard
        max, sum-exp, winner score, id, logit) instead of B x V/tp logits --
        at TP4 70B, B 256 that is 20 KB per rank instead of 16 MB.  Exact: the
        same race as the single-GPU sampler over the same per-token noise."""
        logits = self._mm(hidden, self.lm_head)
        part = ops.sample_partial(logits, self.tp.rank * self.vocab_local, temperature, seeds, offsets)
        return ops.combine_sampled_parts(self.tp.gather_rows(part), out_tokens, out_logprobs)
