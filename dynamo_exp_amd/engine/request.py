"""Engine-side request state and sampling parameters."""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field
from typing import Any, Callable


@dataclass
class SamplingParams:
    temperature: float = 0.0  # 0 = greedy
    top_k: int = 0  # 0 = disabled
    top_p: float = 1.0
    min_p: float = 0.0
    seed: int | None = None
    max_tokens: int = 16
    min_tokens: int = 0
    stop_token_ids: list[int] = field(default_factory=list)  # hidden stop ids (EOS merged in)
    ignore_eos: bool = False
    repetition_penalty: float = 1.0
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    logprobs: bool = False
    # eviction rank of this request's cached blocks once released (reference
    # kv/reuse.rs priority: lower is evicted first)
    cache_priority: int = 0

    @property
    def needs_penalties(self) -> bool:
        return self.repetition_penalty != 1.0 or self.frequency_penalty != 0.0 or self.presence_penalty != 0.0

    @classmethod
    def from_preprocessed(cls, req: dict, eos_token_ids: list[int] | None = None) -> "SamplingParams":
        """Build from a PreprocessedRequest-shaped dict (see llm.protocols)."""
        so = req.get("sampling_options") or {}
        sc = req.get("stop_conditions") or {}
        stop_ids = list(sc.get("stop_token_ids_hidden") or [])
        ignore_eos = bool(sc.get("ignore_eos") or False)
        eos = req.get("eos_token_ids") or eos_token_ids or []
        if not ignore_eos:
            stop_ids = list(dict.fromkeys(stop_ids + list(eos)))
        temp = so.get("temperature")
        if so.get("greed_sampling") or so.get("greedy"):
            temp = 0.0
        return cls(
            temperature=float(temp) if temp is not None else 0.0,
            top_k=int(so.get("top_k") or 0) if (so.get("top_k") or 0) > 0 else 0,
            top_p=float(so.get("top_p") if so.get("top_p") is not None else 1.0),
            min_p=float(so.get("min_p") or 0.0),
            seed=so.get("seed"),
            max_tokens=int(sc.get("max_tokens") or 16),
            min_tokens=int(sc.get("min_tokens") or 0),
            stop_token_ids=stop_ids,
            ignore_eos=ignore_eos,
            repetition_penalty=float(so.get("repetition_penalty") or 1.0),
            frequency_penalty=float(so.get("frequency_penalty") or 0.0),
            presence_penalty=float(so.get("presence_penalty") or 0.0),
            logprobs=bool(req.get("output_options", {}).get("logprobs")) if isinstance(req.get("output_options"), dict) else False,
            cache_priority=int(so.get("cache_priority") or req.get("cache_priority") or 0),
        )


class Status(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    REMOTE_PREFILLING = "remote_prefilling"  # decode side: KV being produced by a prefill worker
    TRANSFERRING = "transferring"  # prefill side: KV being sent to the decode worker
    READING = "reading"  # prefill side: pulling a cached prompt prefix from the decode worker
    FINISHED = "finished"


class FinishReason(str, enum.Enum):
    STOP = "stop"  # hidden stop token / eos
    LENGTH = "length"
    CANCELLED = "cancelled"
    ERROR = "error"
    REMOTE_DECODE = "remote_decode"  # prefill worker handed off to decode


@dataclass
class Request:
    request_id: str
    prompt: list[int]
    params: SamplingParams
    output: list[int] = field(default_factory=list)
    logprobs: list[float] = field(default_factory=list)
    block_ids: list[int] = field(default_factory=list)
    num_computed: int = 0  # tokens whose KV is in the cache
    num_prefix_hit: int = 0  # prompt tokens served from the prefix cache
    block_hashes: list[int] = field(default_factory=list)  # local hashes of registered blocks
    seq_hashes: list[int] = field(default_factory=list)  # sequence hashes of registered blocks
    status: Status = Status.WAITING
    finish_reason: FinishReason | None = None
    arrival: float = field(default_factory=time.perf_counter)
    sched_arrival: float = 0.0  # Scheduler.clock() when queued (deterministic across TP ranks)
    admit_time: float | None = None  # got KV blocks (left the waiting queue)
    first_token_time: float | None = None
    finish_time: float | None = None
    # disaggregation
    remote_prefill: bool = False  # decode side: prefill happens elsewhere
    remote_decode: bool = False  # prefill side: hand the KV to a decode worker
    remote_meta: dict[str, Any] = field(default_factory=dict)
    # prefill side of disaggregation: prompt blocks the decode worker already
    # holds (its prefix-cache hit); pulled instead of recomputed when the local
    # cache has fewer (disagg READ path)
    remote_read_blocks: int = 0
    read_upto: int = 0  # blocks being pulled: [num_computed // bs, read_upto)
    kv_ready: bool = False  # prefill-first policy: blocks allocated, prefix pulled
    # delivery
    on_output: Callable[["Request", list[int], list[float], bool], None] | None = None
    sent: int = 0  # output tokens already delivered
    # asynchronous scheduling: trailing entries of `output` that are
    # placeholders for tokens sampled on the device but not yet read back
    pending: int = 0
    epoch: int = 0  # bumped on preemption: stale pending tokens are dropped
    cancelled: bool = False
    sample_offset: int = 0  # RNG counter for seeded sampling
    # multimodal: embeddings [n, hidden] that replace the prompt tokens at
    # mm_positions (in order); hash_prompt = prompt with those tokens replaced
    # by image-content-derived ids, used for every KV block hash
    mm_embeds: Any = None
    mm_positions: list[int] = field(default_factory=list)
    hash_prompt: list[int] | None = None

    @property
    def num_tokens(self) -> int:
        return len(self.prompt) + len(self.output)

    def all_tokens(self) -> list[int]:
        return self.prompt + self.output

    def hash_tokens(self) -> list[int]:
        """Token ids the KV block hashes are computed over."""
        return (self.hash_prompt if self.hash_prompt is not None else self.prompt) + self.output

    @property
    def finished(self) -> bool:
        return self.status == Status.FINISHED
