"""The first-party MI355X LLM engine (synchronous core + asyncio front).

`LLMEngine` owns model, paged KV, scheduler and runner; `step()` runs one
prefill or decode iteration.  `AsyncLLMEngine` drives `step()` on a dedicated
thread and exposes the token-level engine ABI used by the serving pipeline:

    async for out in engine.generate(preprocessed_request, ctx):  # LLMEngineOutput dicts
        ...

which is the same contract as the reference's `ExecutionContext` engines
(`lib/llm/src/backend.rs:59`, `lib/llm/src/protocols/common/llm_backend.rs:60`).
It also produces the worker load metrics (`ForwardPassMetrics`,
`lib/llm/src/kv_router/protocols.rs:43`) and the KV events for the router.
"""
from __future__ import annotations

import asyncio
import logging
import os
import sys
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, AsyncIterator, Callable

import torch

from ..models.config import ModelConfig, get_config
from ..models.llama import LlamaForCausalLM, TPGroup
from ..runtime.chan import Chan
from ..utils import streams, tracing
from ..utils.faults import FAULTS
from .kv_manager import KVEvent, KVManager
from .model_runner import ModelRunner, RunnerConfig
from .request import FinishReason, Request, SamplingParams, Status
from .scheduler import Batch, Scheduler, SchedulerConfig

log = logging.getLogger("dynamo_exp_amd.engine")
# DX_SLOW_REQUEST_S=<seconds>: log the phase breakdown of requests whose TTFT exceeds it
_SLOW_REQ_S = float(os.environ.get("DX_SLOW_REQUEST_S", "0") or 0)


from .policy import PREFILL_ENGINE_DEFAULTS, SERVING_DEFAULTS  # noqa: E402,F401 -- re-exported


@dataclass
class EngineConfig:
    model: str = "llama3-8b"  # preset name or HF dir
    random_init: bool = True
    seed: int = 0
    block_size: int = 64
    max_model_len: int = 8192
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 16384
    max_prefill_streak: int = 4
    chunked_prefill: bool = True
    min_prefill_tokens: int = 0  # prefill batching (scheduler.SchedulerConfig)
    max_prefill_delay: float = 0.0
    prefill_hold_min_decode: int = 0  # hold prompts only while >= this many streams decode
    prefill_hold_partial: int = 0  # >= this many decoding streams: the hold also covers a split prompt's remainder
    prefill_whole_prompts: bool = False  # past half the budget, do not split a new prompt
    gpu_memory_utilization: float = 0.90
    num_gpu_blocks: int | None = None
    enable_prefix_caching: bool = True
    use_cuda_graph: bool = True
    graph_sizes: tuple | None = None
    device: str = "cuda"
    tp_size: int = 1
    host_kv_blocks: int = 0  # pinned-host KV offload tier size (blocks); -1 = sized from free host RAM
    quantization: str | None = None  # None (bf16) | "fp8" (w8a8 e4m3fn linears)
    # KV cache element type: "auto" (bf16) | "fp8" (OCP e4m3fn, per-tensor
    # scales kv_scales; halves the KV bytes decode attention streams)
    kv_cache_dtype: str = "auto"
    kv_scales: tuple = (1.0, 1.0)
    # the KV cache is written by peer processes (decode engine behind the
    # one-sided "ipc" KV transport): allocate it shareable (disagg/kv_share.py)
    kv_shared: bool = os.environ.get("DX_KV_SHARED", "0") == "1"
    # TP > 1 random init: every rank takes its shard of ONE full random model
    # (seed `seed`), so a TP engine computes exactly the TP = 1 model (token
    # checks across layouts); default: independent per-rank shards (cheaper)
    shard_consistent_init: bool = False
    # pure-decode steps with nothing waiting run this many graph replays per
    # host round trip (device-side token feedback, decode_advance kernel).
    # Off by default: measured no throughput gain (the per-token bookkeeping
    # still runs with the GPU idle, just once per k steps) and +30 ms TTFT p50
    # in the aggregated bench (profiles/README.md, "multi-step decode").
    multi_step: int = int(os.environ.get("DX_MULTI_STEP", "1"))
    # asynchronous scheduling: step t+1 is scheduled and enqueued before step
    # t's sampled tokens are read back (decode inputs patched on the device),
    # so host bookkeeping overlaps the GPU instead of idling it
    async_schedule: bool = os.environ.get("DX_ASYNC_SCHEDULE", "1") != "0"

    @classmethod
    def from_args(cls, **kw) -> "EngineConfig":
        names = set(cls.__dataclass_fields__)
        return cls(**{k: v for k, v in kw.items() if k in names and v is not None})


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model_cfg: ModelConfig | None = None, tp: TPGroup | None = None,
                 model: LlamaForCausalLM | None = None):
        self.cfg = cfg
        self.model_cfg = model_cfg or get_config(cfg.model)
        if cfg.max_model_len > self.model_cfg.max_position_embeddings:
            cfg.max_model_len = self.model_cfg.max_position_embeddings
        dev = torch.device(cfg.device)
        if model is None:
            model = LlamaForCausalLM(self.model_cfg, device=dev, tp=tp)
            if cfg.random_init or not os.path.isdir(cfg.model):
                model.random_init(cfg.seed)
            else:
                model.load_safetensors(cfg.model)
            if cfg.quantization == "fp8":
                model.quantize_fp8()
            elif cfg.quantization:
                raise ValueError(f"unsupported quantization {cfg.quantization!r} (supported: fp8)")
        self.model = model
        self._cuda = model.device.type == "cuda"
        if model.device.type == "cuda" and not model.fp8:
            model.enable_fused_mlp()  # prefill MLPs on the fused SwiGLU GEMM (csrc/kernels/gemm256.hip)
        model.fold_norms()  # norm weights into the projections: large forwards skip the norm kernels
        if cfg.kv_cache_dtype not in ("auto", "bf16", "bfloat16", "fp8", "fp8_e4m3"):
            raise ValueError(f"unsupported kv_cache_dtype {cfg.kv_cache_dtype!r} (supported: auto, fp8)")
        kv_fp8 = cfg.kv_cache_dtype.startswith("fp8")
        model.kv_scales = tuple(float(x) for x in cfg.kv_scales) if kv_fp8 else (1.0, 1.0)
        rcfg = RunnerConfig(block_size=cfg.block_size, num_gpu_blocks=cfg.num_gpu_blocks,
                            gpu_memory_utilization=cfg.gpu_memory_utilization, max_model_len=cfg.max_model_len,
                            max_num_seqs=cfg.max_num_seqs, use_cuda_graph=cfg.use_cuda_graph,
                            kv_dtype=torch.float8_e4m3fn if kv_fp8 else torch.bfloat16, kv_shared=cfg.kv_shared)
        if cfg.graph_sizes:
            rcfg.graph_sizes = tuple(cfg.graph_sizes)
        self.runner = ModelRunner(model, rcfg)
        self.gemm_report: list[dict] = []
        self.prefill_gemm_report: list[dict] = []
        self._event_listeners: list[Callable[[list[KVEvent]], None]] = []
        self.host_tier = None
        if cfg.host_kv_blocks and cfg.enable_prefix_caching:
            from .host_tier import HostKVTier, auto_host_blocks

            n = cfg.host_kv_blocks
            if n < 0:
                kvc = self.runner.kv_cache
                n = auto_host_blocks(kvc[:, :, :1].numel() * kvc.element_size(), self.runner.num_blocks)
                log.info("host KV tier: %d blocks (auto)", n)
            if n > 0:
                self.host_tier = HostKVTier(self.runner.kv_cache, n)
        self.kv = KVManager(self.runner.num_blocks, cfg.block_size, cfg.enable_prefix_caching, self._emit_events,
                            host_tier=self.host_tier)
        self.scheduler = Scheduler(
            SchedulerConfig(max_num_seqs=cfg.max_num_seqs, max_num_batched_tokens=cfg.max_num_batched_tokens,
                            max_model_len=cfg.max_model_len, max_prefill_streak=cfg.max_prefill_streak,
                            chunked_prefill=cfg.chunked_prefill, min_prefill_tokens=cfg.min_prefill_tokens,
                            max_prefill_delay=cfg.max_prefill_delay,
                            prefill_hold_min_decode=cfg.prefill_hold_min_decode,
                            prefill_hold_partial=cfg.prefill_hold_partial,
                            prefill_whole_prompts=cfg.prefill_whole_prompts), self.kv)
        self.requests: dict[str, Request] = {}
        self.stats = dict(steps=0, prefill_steps=0, decode_steps=0, mixed_steps=0, prompt_tokens=0,
                          generated_tokens=0, prefill_step_tokens=0)
        # DX_STEP_SIZES=1: (tokens, prompts) of every prefill / mixed step, for
        # studies of the step-size distribution (tools, bench stderr)
        self.step_sizes: list | None = [] if os.environ.get("DX_STEP_SIZES") == "1" else None
        self.eos_token_ids = list(self.model_cfg.eos_token_id)
        self.prefill_done_hook: Callable[[Request], None] | None = None  # disagg prefill worker
        # disagg prefill worker: called with each scheduled batch before its
        # forward (announce the requests whose KV streams out during it)
        self.batch_hook: Callable[[Batch], None] | None = None
        self.last_batch: Batch | None = None
        self._inflight = None  # async scheduling: (batch, runner.Launched) not read back yet
        self.timing = {"schedule": 0.0, "execute": 0.0, "update": 0.0, "deliver": 0.0}
        self.request_timer = tracing.RequestTimer()

    # ---------------------------------------------------------------- events
    def add_kv_event_listener(self, fn: Callable[[list[KVEvent]], None]) -> None:
        self._event_listeners.append(fn)

    def _emit_events(self, evs: list[KVEvent]) -> None:
        for fn in self._event_listeners:
            try:
                fn(evs)
            except Exception:  # pragma: no cover
                log.exception("kv event listener failed")

    # ---------------------------------------------------------------- fp8 KV
    @torch.no_grad()
    def calibrate_kv_scales(self, prompts: list[list[int]], margin: float = 1.0) -> tuple[float, float]:
        """Per-tensor scales of an fp8 KV cache from calibration prompts
        (vLLM's calculate_kv_scales role): run their prefill, take the largest
        |K| and |V| (post-RoPE, as cached) over all layers, and map it to
        e4m3's largest normal (scale = amax * margin / 448).  Sets and returns
        the scales.

        Every cached KV block -- device and host tier -- was quantised with
        the OLD scales (the calibration prompts' own blocks included), so the
        prefix caches are dropped before and after (Removed events reach the
        router), and decode graphs captured earlier, which carry the scales as
        kernel arguments, are captured again.  Needs an idle engine."""
        if not self.cfg.kv_cache_dtype.startswith("fp8"):
            raise ValueError("calibrate_kv_scales needs kv_cache_dtype='fp8'")
        if self.has_unfinished():
            raise RuntimeError("calibrate_kv_scales needs an idle engine (requests in flight use the old scales)")
        if getattr(self, "kv_transfer_attached", False):
            # peers validated (and cached) this engine's published scales when
            # they first reached it; new scales would make them decode its e4m3
            # bytes with the old ones
            raise RuntimeError("calibrate_kv_scales before attaching a KV transfer agent (its peers hold the "
                               "published kv_scales); pass the calibrated scales to every worker instead")
        m = self.model
        self.kv.reset_prefix_cache()  # no prefix hits: every calibration token is written (and measured)
        m.kv_amax = torch.zeros(2, device=m.device)
        try:
            for i, p in enumerate(prompts):
                rid = f"__kv_calib_{i}"
                self.add_request(rid, list(p), SamplingParams(max_tokens=1, ignore_eos=True))
            while self.has_unfinished():
                self.step()
            amax = m.kv_amax.tolist()
        finally:
            m.kv_amax = None
        scales = tuple(max(a * margin / 448.0, 1e-6) for a in amax)
        m.kv_scales = scales
        self.cfg.kv_scales = scales
        self.kv.reset_prefix_cache()  # the calibration prompts' blocks hold old-scale bytes
        if self.runner.graphs:
            self.runner.graphs.clear()
            self.runner.graphs_sharded.clear()
            self.runner.capture_graphs()
        return scales

    # ---------------------------------------------------------------- requests
    def warmup(self) -> float:
        """Before serving: load the prefill GEMM kernels for the chunk sizes the
        scheduler produces (powers of two up to the token budget) and capture
        the decode graphs."""
        t0 = time.perf_counter()
        streams.enter_compute(self.model.device)
        streams.log_plan(self.model.device)
        if self.model.device.type == "cuda" and self.model.layers:
            T = 16
            while T <= self.cfg.max_num_batched_tokens:
                self.model.warmup_linears(T)
                T *= 2
            # prefill-size projections: hipBLASLt's slow M windows -> gemm256
            self.prefill_gemm_report = self.model.tune_prefill_gemms(
                min(self.cfg.max_num_batched_tokens, self.cfg.max_num_seqs * self.cfg.max_model_len)
                + self.cfg.max_num_seqs)
            log.info("prefill GEMM: %d of %d (bucket, projection) pairs on gemm256",
                     sum(r["adopted"] for r in self.prefill_gemm_report), len(self.prefill_gemm_report))
            if self.runner.cfg.use_cuda_graph:
                # decode batch sizes: hand-written small-M GEMM where it beats the library
                # (w8a8 models: hipBLASLt's fp8 GEMMs, no hand-kernel candidates)
                self.gemm_report = [] if self.model.fp8 else self.model.tune_gemms(self.runner.cfg.graph_sizes)
                n = sum(r["adopted"] for r in self.gemm_report)
                log.info("small-M GEMM: %d of %d decode GEMM shapes on the MFMA kernel", n, len(self.gemm_report))
            torch.cuda.synchronize(self.model.device)
        return self.runner.capture_graphs() + (time.perf_counter() - t0)

    def add_request(self, request_id: str | None, prompt: list[int], params: SamplingParams,
                    on_output=None, remote_prefill: bool = False, remote_decode: bool = False,
                    remote_meta: dict | None = None, mm_embeds=None, mm_hash: int | None = None,
                    remote_read_blocks: int = 0) -> Request:
        """`remote_read_blocks` (prefill worker): leading prompt blocks the
        decode worker already caches -- pulled instead of recomputed when the
        local prefix cache has fewer (scheduler.on_remote_read).
        `mm_embeds` ([n, hidden] tensor) replace the prompt's image
        placeholder tokens (model_cfg.image_token_id), in order; `mm_hash`
        identifies the image content for prefix caching (derived from the
        embeddings when omitted)."""
        rid = request_id or uuid.uuid4().hex
        remote_read_blocks = remote_read_blocks or int((remote_meta or {}).get("read_blocks", 0))
        if not params.ignore_eos:
            params.stop_token_ids = list(dict.fromkeys(list(params.stop_token_ids) + self.eos_token_ids))
        req = Request(rid, list(prompt), params, on_output=on_output, remote_prefill=remote_prefill,
                      remote_decode=remote_decode, remote_meta=remote_meta or {},
                      remote_read_blocks=remote_read_blocks)
        if mm_embeds is not None:
            self._attach_mm(req, mm_embeds, mm_hash)
        self.requests[rid] = req
        self.scheduler.add(req)
        self.stats["prompt_tokens"] += len(prompt)
        return req

    def _attach_mm(self, req: Request, embeds, mm_hash: int | None) -> None:
        tok = self.model_cfg.image_token_id
        if tok is None:
            raise ValueError(f"{self.model_cfg.name} has no image token; multimodal input unsupported")
        pos = [i for i, t in enumerate(req.prompt) if t == tok]
        embeds = embeds.reshape(-1, embeds.shape[-1])
        if len(pos) != embeds.shape[0]:
            raise ValueError(f"{len(pos)} image placeholder tokens but {embeds.shape[0]} image embeddings")
        if mm_hash is None:
            from ..kv.hashing import xxh3_64

            mm_hash = xxh3_64(embeds.detach().to("cpu", torch.float32).numpy().tobytes(), 0)
        req.mm_embeds = embeds.to(self.model.device, self.model.dtype)
        req.mm_positions = pos
        hp = list(req.prompt)
        for k, i in enumerate(pos):  # image-content ids in the top half of u32 space
            hp[i] = 0x80000000 | ((mm_hash + k) & 0x7FFFFFFF)
        req.hash_prompt = hp

    def abort(self, request_id: str) -> None:
        r = self.requests.get(request_id)
        if r is not None:
            r.cancelled = True
            if self.scheduler.abort(request_id) is not None:
                self._deliver(r)

    def has_unfinished(self) -> bool:
        return self.scheduler.num_unfinished() > 0 or self._inflight is not None

    def has_pending_work(self) -> bool:
        """Whether step() would do anything now."""
        return self.scheduler.has_work() or self._inflight is not None

    # ---------------------------------------------------------------- step
    def step(self) -> list[Request]:
        if self._cuda:  # this thread's launches go to the high-priority compute stream (utils/streams.py)
            streams.enter_compute(self.model.device)
        if self.cfg.async_schedule and self.cfg.multi_step <= 1:
            return self._step_async()
        pc = time.perf_counter
        t0 = pc()
        batch = self.scheduler.schedule()
        self.kv.maintain()
        t1 = pc()
        self.timing["schedule"] += t1 - t0
        if batch is None:
            return []
        self.last_batch = batch
        FAULTS.on_engine_step()
        if self.batch_hook is not None:
            self.batch_hook(batch)
        k = 1
        if batch.kind == "decode" and self.cfg.multi_step > 1 and self.runner.supports_multi_step(batch.requests):
            k = self.scheduler.reserve_multi(batch, self.cfg.multi_step)
        res = None
        if k > 1:
            with tracing.span("engine.step/decode_multi"):
                res = self.runner.execute_decode_multi(batch.requests, k)
        if res is not None:
            t2 = pc()
            self.timing["execute"] += t2 - t1
            out = self.scheduler.update_multi(batch, res[0], res[1])
            n_steps = k
        else:
            with tracing.span(f"engine.step/{batch.kind}"):
                toks, lps = self.runner.execute(batch)
            t2 = pc()
            self.timing["execute"] += t2 - t1
            out = self.scheduler.update(batch, toks, lps)
            n_steps = 1
        t3 = pc()
        self.timing["update"] += t3 - t2
        self.stats["steps"] += n_steps
        self.stats[f"{batch.kind}_steps"] += n_steps
        if batch.kind != "decode":
            self.stats["prefill_step_tokens"] += batch.num_tokens
            if self.step_sizes is not None:
                self.step_sizes.append((batch.num_tokens, batch.n_prefill))
        now = time.perf_counter()
        for r in out:
            if r.first_token_time is None:
                r.first_token_time = now
            if r.status == Status.TRANSFERRING:
                if self.prefill_done_hook is not None:
                    self.prefill_done_hook(r)
                continue
            self.stats["generated_tokens"] += len(r.output) - r.sent
            self._deliver(r)
        t4 = pc()
        self.timing["deliver"] += t4 - t3
        if _SLOW_REQ_S and t4 - t0 > _SLOW_REQ_S:
            log.warning("slow step %s: schedule %.3fs execute %.3fs update %.3fs deliver %.3fs; rows %s",
                        batch.kind, t1 - t0, t2 - t1, t3 - t2, t4 - t3,
                        [(len(r.prompt), n) for r, n in zip(batch.requests, batch.num_new)][:24])
        return out

    # ---------------------------------------------------------------- async step
    def _step_async(self) -> list[Request]:
        """Schedule + enqueue step t+1, then read back and apply step t (the
        GPU runs t+1 meanwhile).  Falls back to resolving the batch in flight
        first when the next batch needs token values on the host (penalties)."""
        pc = time.perf_counter
        t0 = pc()
        prev = self._inflight
        if prev is not None and any(r.params.needs_penalties for r in self.scheduler.running):
            self._inflight = None
            return self._apply_launched(prev, t0)
        batch = self.scheduler.schedule()
        self.kv.maintain()
        t1 = pc()
        self.timing["schedule"] += t1 - t0
        launched = None
        if batch is not None:
            self.last_batch = batch
            FAULTS.on_engine_step()
            if self.batch_hook is not None:
                self.batch_hook(batch)
            with tracing.span(f"engine.step/{batch.kind}"):
                h = self.runner.launch(batch, prev[1] if prev is not None else None)
            self.scheduler.pre_update(batch)
            launched = (batch, h)
        self.timing["execute"] += pc() - t1
        self._inflight = launched
        if prev is None:
            return []
        return self._apply_launched(prev, pc())

    def _apply_launched(self, launched, t0: float) -> list[Request]:
        pc = time.perf_counter
        batch, h = launched
        toks, lps = self.runner.fetch(h)
        t2 = pc()
        self.timing["execute"] += t2 - t0
        out = self.scheduler.update_async(batch, toks, lps)
        t3 = pc()
        self.timing["update"] += t3 - t2
        self.stats["steps"] += 1
        self.stats[f"{batch.kind}_steps"] += 1
        if batch.kind != "decode":
            self.stats["prefill_step_tokens"] += batch.num_tokens
            if self.step_sizes is not None:
                self.step_sizes.append((batch.num_tokens, batch.n_prefill))
        now = pc()
        for r in out:
            if r.first_token_time is None:
                r.first_token_time = now
            if r.status == Status.TRANSFERRING:
                if self.prefill_done_hook is not None:
                    self.prefill_done_hook(r)
                continue
            self.stats["generated_tokens"] += len(r.output) - r.pending - r.sent
            self._deliver(r)
        self.timing["deliver"] += pc() - t3
        return out

    def _deliver(self, r: Request) -> None:
        end = len(r.output) - r.pending  # placeholders of tokens still in flight stay back
        new = r.output[r.sent:end]
        lps = r.logprobs[r.sent:end]
        r.sent = end
        fin = r.finished
        if r.on_output is not None and (new or fin):
            r.on_output(r, new, lps, fin)
        if fin:
            self.requests.pop(r.request_id, None)
            self.request_timer.observe(r)
            if _SLOW_REQ_S and r.first_token_time is not None and r.first_token_time - r.arrival > _SLOW_REQ_S:
                adm = getattr(r, "admit_time", None)
                log.warning("slow request %s: ttft %.3fs (queued %.3fs, prefill %.3fs), prompt %d, preempted %d, "
                            "running %d waiting %d free blocks %d", r.request_id, r.first_token_time - r.arrival,
                            (adm - r.arrival) if adm else -1, (r.first_token_time - adm) if adm else -1, len(r.prompt),
                            getattr(r, "preempted", 0), self.scheduler.num_active(), len(self.scheduler.waiting),
                            self.kv.num_free())

    # ---------------------------------------------------------------- disagg hooks
    def finish_remote_prefill(self, request_id: str, first_token: int | None, logprob: float = 0.0) -> None:
        r = self.scheduler.finish_remote_prefill(request_id, first_token, logprob)
        if r is not None:
            if r.first_token_time is None:
                r.first_token_time = time.perf_counter()
            self.stats["generated_tokens"] += 1 if first_token is not None else 0
            self._deliver(r)

    def fallback_local_prefill(self, request_id: str) -> bool:
        """Decode side: prefill a remote-prefill request locally after all
        (its transfer never started: disagg/agent.py decode_leader_hook)."""
        return self.scheduler.fallback_local(request_id) is not None

    def finish_remote_read(self, request_id: str, ok: bool = True) -> None:
        """Prefill worker: a pulled prompt prefix landed (READ path); ok=False:
        its bytes are not the prefix (scheduler.finish_remote_read)."""
        self.scheduler.finish_remote_read(request_id, ok)

    def finish_transfer(self, request_id: str) -> None:
        r = self.scheduler.finish_transfer(request_id)
        if r is not None:
            self._deliver(r)

    # ---------------------------------------------------------------- metrics
    def forward_pass_metrics(self) -> dict[str, Any]:
        """Same fields as the reference ForwardPassMetrics."""
        s = self.scheduler
        total = self.kv.num_blocks
        used = total - self.kv.num_free()
        return dict(
            request_active_slots=s.num_active(),
            request_total_slots=self.cfg.max_num_seqs,
            kv_active_blocks=used,
            kv_total_blocks=total,
            num_requests_waiting=len(s.waiting),
            gpu_cache_usage_perc=used / max(1, total),
            gpu_prefix_cache_hit_rate=self.kv.hit_rate(),
        )


def _dispatch(items: list) -> None:
    for q, item in items:
        q.put_nowait(item)


class AsyncLLMEngine:
    """Runs an LLMEngine on its own thread; asyncio-facing token-level API."""

    def __init__(self, engine: LLMEngine, idle_sleep: float = 0.0005):
        self.engine = engine
        self._lock = threading.Lock()
        self._pending: list[tuple] = []  # (fn, args) executed on the engine thread
        self._wake = threading.Event()
        self._stop = False
        self._idle_sleep = idle_sleep
        self._thread = threading.Thread(target=self._loop, name="dx-engine", daemon=True)
        self._started = False
        self.step_hooks: list[Callable[[], None]] = []  # run on the engine thread each iteration
        # outputs produced during one engine iteration, handed to each event
        # loop with ONE call_soon_threadsafe (one self-pipe wakeup per step
        # instead of one per stream)
        self._outbox: dict[Any, list] = {}

    def start(self) -> "AsyncLLMEngine":
        if not self._started:
            self._started = True
            # The engine thread drops the GIL while it waits on the GPU; with
            # the default 5 ms switch interval it can then wait up to 5 ms per
            # wait to get it back from a busy event loop.  0.5 ms bounds that.
            sw = float(os.environ.get("DX_GIL_SWITCH_INTERVAL_S", "0.0005"))
            if sw > 0 and sys.getswitchinterval() > sw:
                sys.setswitchinterval(sw)
            self._thread.start()
        return self

    def shutdown(self) -> None:
        self._stop = True
        self._wake.set()
        if self._started:
            self._thread.join(timeout=10)

    def call(self, fn, *args) -> None:
        """Run fn(*args) on the engine thread before the next step."""
        with self._lock:
            self._pending.append((fn, args))
        self._wake.set()

    def _stats_line(self, st: dict) -> None:
        """DX_ENGINE_STATS_S=<s>: every s seconds log the device-busy fraction
        (GPU time of the launches / wall) and the host phases of the engine
        loop -- how a serving process compares with bench.py's driver loop."""
        eng = getattr(self.engine, "engine", self.engine)
        runner = getattr(eng, "runner", None)
        if runner is None:
            return
        runner.harvest_gpu_time()
        now = time.perf_counter()
        cur = {"gpu": runner.timing["prefill_gpu"] + runner.timing["decode_gpu"],
               "tokens": eng.stats.get("generated_tokens", 0), "steps": eng.stats.get("steps", 0),
               **{k: eng.timing.get(k, 0.0) for k in ("schedule", "execute", "update", "deliver")}}
        if st:
            dt = now - st["t"]
            log.info("engine stats over %.1fs: device busy %.3f, %.0f tok/s, %d steps, host ms/step %s", dt,
                     (cur["gpu"] - st["gpu"]) / dt, (cur["tokens"] - st["tokens"]) / dt, cur["steps"] - st["steps"],
                     {k: round((cur[k] - st[k]) * 1e3 / max(1, cur["steps"] - st["steps"]), 3)
                      for k in ("schedule", "execute", "update", "deliver")})
        st.update(cur, t=now)

    def _loop(self) -> None:
        eng = self.engine
        dev = eng.model.device
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        period = float(os.environ.get("DX_ENGINE_STATS_S", "0") or 0)
        st: dict = {}
        t_stats = time.perf_counter()
        while not self._stop:
            if period and time.perf_counter() - t_stats >= period:
                t_stats = time.perf_counter()
                try:
                    self._stats_line(st)
                except Exception:  # noqa: BLE001 -- diagnostics only
                    log.exception("engine stats failed")
            with self._lock:
                pend, self._pending = self._pending, []
            for fn, args in pend:
                try:
                    fn(*args)
                except Exception:
                    log.exception("engine call failed")
            for h in self.step_hooks:
                try:
                    h()
                except Exception:
                    log.exception("step hook failed")
            has_work = eng.has_pending_work() if hasattr(eng, "has_pending_work") else eng.scheduler.has_work()
            if has_work:
                try:
                    eng.step()
                except Exception:
                    log.exception("engine step failed")
                    for r in list(eng.requests.values()):
                        eng.scheduler.abort(r.request_id)
                        r.finish_reason = FinishReason.ERROR
                        eng._deliver(r)
                self._flush()
            else:
                self._flush()
                self._wake.wait(timeout=0.05 if not self.step_hooks else self._idle_sleep)
                self._wake.clear()

    def _post(self, loop, q, item) -> None:
        box = self._outbox.get(loop)
        if box is None:
            box = self._outbox[loop] = []
        box.append((q, item))

    def _flush(self) -> None:
        if not self._outbox:
            return
        boxes, self._outbox = self._outbox, {}
        for loop, items in boxes.items():
            try:
                loop.call_soon_threadsafe(_dispatch, items)
            except RuntimeError:  # loop closed: its consumers are gone
                pass

    async def generate(self, request_id: str | None, prompt: list[int], params: SamplingParams,
                       remote_prefill: bool = False, remote_decode: bool = False,
                       remote_meta: dict | None = None, context=None, mm_embeds=None,
                       mm_hash: int | None = None) -> AsyncIterator[dict]:
        """Yield LLMEngineOutput dicts: {token_ids, cum_log_probs, log_probs, finish_reason}."""
        loop = asyncio.get_running_loop()
        q = Chan()
        rid = request_id or uuid.uuid4().hex

        def on_output(req, toks, lps, fin):
            reason = req.finish_reason.value if (fin and req.finish_reason) else None
            item = {"token_ids": list(toks), "log_probs": list(lps), "finish_reason": reason}
            if threading.current_thread() is self._thread:
                self._post(loop, q, item)
            else:  # delivered outside the engine loop (tests driving step() directly)
                loop.call_soon_threadsafe(q.put_nowait, item)

        self.call(self.engine.add_request, rid, prompt, params, on_output, remote_prefill, remote_decode,
                  remote_meta, mm_embeds, mm_hash)
        try:
            while True:
                item = await q.get()
                yield item
                if item["finish_reason"] is not None:
                    return
                if context is not None and getattr(context, "is_stopped", lambda: False)():
                    self.call(self.engine.abort, rid)
                    return
        except (asyncio.CancelledError, GeneratorExit):
            self.call(self.engine.abort, rid)
            raise
