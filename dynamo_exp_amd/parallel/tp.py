"""Tensor parallelism: one process per GPU, SPMD engines kept in lockstep.

Every TP rank runs a full LLMEngine over its weight shard (Megatron-style
column/row split, see models/llama.py) and the same deterministic scheduler /
block manager.  Only the leader (rank 0) receives requests; at the start of
each step it publishes the step's input *events* (new requests, aborts, KV
transfer events) and its step clock on the node-local event plane -- a
shared-memory broadcast ring (csrc/runtime/event_ring.h; gloo broadcast only
as a fallback) -- and every rank applies them in the same order and steps.
Because sampling runs on all-gathered (bit-identical) logits with identical
seeds, all ranks pick the same tokens and their schedulers never diverge --
no per-step tensor broadcast of batch metadata is needed.  Activation
all-reduces go over RCCL (xGMI), captured inside the decode hipGraphs.

(The reference delegates TP to vLLM/SGLang: lib/engines/vllm0_8/src/lib.rs:371,
lib/engines/sglang/src/worker.rs:286-345.)
"""
from __future__ import annotations

import dataclasses
import datetime
import logging
import os
import threading
import time

import msgpack
import torch
import torch.distributed as dist

from ..engine.engine import EngineConfig, LLMEngine
from ..engine.request import SamplingParams
from ..models.config import get_config
from ..models.llama import LlamaForCausalLM, TPGroup
from ..utils import streams

log = logging.getLogger("dynamo_exp_amd.tp")

LONG = datetime.timedelta(days=7)


class EventPlane:
    """Leader -> follower step events, msgpack-encoded.  `shm` (default): a
    native shared-memory broadcast ring, one publish per step, followers
    block in native code with the GIL released; `gloo`: broadcast_object_list
    over the CPU group (DX_TP_EVENTS=gloo, or no native runtime)."""

    SLOTS, SLOT_BYTES = 64, 1 << 20

    def __init__(self, group, rank: int, world: int):
        import uuid

        from .. import _native

        self.group, self.rank, self.world = group, rank, world
        self.ring = None
        rt = _native.runtime()
        name = [None]
        if rank == 0 and rt is not None and os.environ.get("DX_TP_EVENTS", "shm") == "shm":
            name[0] = f"/dx_tp_{os.getpid()}_{uuid.uuid4().hex[:12]}"
            self.ring = rt.EventRing.create(name[0], self.SLOTS, self.SLOT_BYTES, world - 1)
        # one-time: the ring's name (or None); group_src: the group may be a
        # sub-group of a larger world (the bench's engines)
        dist.broadcast_object_list(name, group_src=0, group=group)
        if rank > 0 and name[0] is not None:
            self.ring = rt.EventRing.attach(name[0], rank - 1)
        self.kind = "shm" if name[0] is not None else "gloo"
        dist.barrier(group=group)
        if rank == 0 and self.ring is not None:
            self.ring.unlink()  # every rank has it mapped; the name is no longer needed

    @staticmethod
    def encode(now: float, events: list) -> bytes:
        wire = []
        for e in events:
            if e[0] == "add":
                _, rid, prompt, params, rp, rd, meta = e
                wire.append(["add", rid, list(prompt), dataclasses.asdict(params), rp, rd, meta])
            else:
                wire.append(list(e))
        return msgpack.packb([now, wire], use_bin_type=True)

    @staticmethod
    def decode(data: bytes):
        now, wire = msgpack.unpackb(data, raw=False, strict_map_key=False)
        out = []
        for e in wire:
            if e[0] == "add":
                _, rid, prompt, params, rp, rd, meta = e
                out.append(("add", rid, prompt, SamplingParams(**params), rp, rd, meta))
            else:
                out.append(tuple(e))
        return now, out

    def publish(self, now: float, events: list) -> None:
        data = self.encode(now, events)
        if self.ring is not None:
            self.ring.publish(data)
        else:
            dist.broadcast_object_list([data], group_src=0, group=self.group)

    def receive(self):
        """Followers: the next step's (now, events); None once the leader closed."""
        if self.ring is not None:
            data = self.ring.poll()
            if data is None:
                return None
        else:
            obj = [None]
            dist.broadcast_object_list(obj, group_src=0, group=self.group)
            data = obj[0]
        return self.decode(data)

    def close(self) -> None:
        if self.ring is not None and self.rank == 0:
            self.ring.close()


class ReplicatedEngine:
    """Wraps an LLMEngine; rank 0 drives, followers mirror.

    Besides requests and aborts, the leader can broadcast named extension
    events (`submit(name, payload)`): every rank runs `handlers[name](payload)`
    before the step, in the same order -- how the disaggregated KV transfer
    posts and completes per-rank receives in lockstep (disagg/agent.py).
    `post_step_hooks` run on every rank after each step.  With world == 1 (no
    group) it is a plain single-process driver with the same API, so serving
    workers use one code path for TP = 1 and TP > 1."""

    def __init__(self, engine: LLMEngine, cpu_group, rank: int, world: int = 1):
        self.engine = engine
        self.group = cpu_group
        self.rank = rank
        self.world = world
        self.pending: list[tuple] = []
        self._lock = threading.Lock()
        self.stopped = False
        self.handlers: dict = {}
        self.post_step_hooks: list = []
        self.followers: list = []  # spawned follower processes (leader only)
        self._now = time.perf_counter()
        self.events = None
        if world > 1:
            engine.scheduler.clock = lambda: self._now
            self.events = EventPlane(cpu_group, rank, world)

    # leader API (same signatures as LLMEngine)
    def add_request(self, request_id, prompt, params: SamplingParams, on_output=None, remote_prefill=False,
                    remote_decode=False, remote_meta=None, mm_embeds=None, mm_hash=None):
        if mm_embeds is not None and self.world > 1:
            raise NotImplementedError("multimodal inputs are not supported with tensor parallelism")
        with self._lock:
            self.pending.append(("add", request_id, list(prompt), params, remote_prefill, remote_decode,
                                 remote_meta, on_output, mm_embeds, mm_hash))

    def abort(self, request_id):
        with self._lock:
            self.pending.append(("abort", request_id))

    def submit(self, name: str, payload) -> None:
        """Run handlers[name](payload) on every rank before the next step."""
        with self._lock:
            self.pending.append(("ext", name, payload))

    def shutdown(self):
        with self._lock:
            self.pending.append(("shutdown",))

    def has_unfinished(self) -> bool:
        return bool(self.pending) or self.engine.has_unfinished()

    def has_pending_work(self) -> bool:
        # the engine's own view includes an asynchronously scheduled batch in flight
        return bool(self.pending) or self.engine.has_pending_work()

    def __getattr__(self, name):
        return getattr(self.engine, name)

    def step(self):
        with self._lock:
            events, self.pending = self.pending, []
        local = {}
        wire = []
        for e in events:
            if e[0] == "add":
                local[e[1]] = (e[7], e[8], e[9])  # callbacks / image embeddings stay on the leader
                wire.append(e[:7])
            else:
                wire.append(e)
        now = time.perf_counter()
        if self.world > 1:
            self.events.publish(now, wire)
            if any(e[0] == "shutdown" for e in wire):
                self.events.close()
        return self._apply_and_step(now, wire, local)

    def _apply_and_step(self, now, events, local):
        # every rank's scheduler sees the leader's step time (prefill-batching
        # hold decisions must not depend on a rank's own clock)
        self._now = now
        if getattr(self.engine, "_cuda", False):  # ext handlers (KV pack / unpack) launch from this thread too
            streams.enter_compute(self.engine.model.device)
        for e in events:
            if e[0] == "add":
                _, rid, prompt, params, rp, rd, meta = e
                cb, mm, mh = local.get(rid, (None, None, None))
                if mm is not None:
                    self.engine.add_request(rid, prompt, params, cb, rp, rd, meta, mm, mh)
                else:
                    self.engine.add_request(rid, prompt, params, cb, rp, rd, meta)
            elif e[0] == "abort":
                self.engine.abort(e[1])
            elif e[0] == "ext":
                self.handlers[e[1]](e[2])
            elif e[0] == "shutdown":
                self.stopped = True
                return []
        out = self.engine.step()
        if self.world > 1:
            self.engine.model.tp.check()  # custom all-reduce barrier timeout -> fail this worker
        for h in self.post_step_hooks:
            h()
        return out

    def release(self) -> None:
        """Drop this rank's IPC mappings of its peers' custom all-reduce
        buffers.  Every rank calls it, then the group barriers, before any
        rank exits: a producer that exits while a peer still maps its buffer
        makes torch warn about live shared CUDA blocks."""
        ar = getattr(self.engine.model.tp, "custom_ar", None)
        if ar is not None:
            ar.close()

    def follower_loop(self) -> None:
        while not self.stopped:
            msg = self.events.receive()
            if msg is None:  # leader closed the event plane
                break
            self._apply_and_step(msg[0], msg[1], {})


def init_tp_group(rank: int, world: int, master: str, port: int, device: torch.device):
    os.environ.setdefault("MASTER_ADDR", master)
    os.environ.setdefault("MASTER_PORT", str(port))
    # DX_TP_BACKEND=gloo: TP ranks that share one GPU (functional GPU tests;
    # RCCL needs one device per rank) -- all-reduces then go through the
    # custom IPC all-reduce or gloo, never captured in graphs
    backend = os.environ.get("DX_TP_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
    dist.init_process_group(backend, rank=rank, world_size=world, init_method=f"tcp://{master}:{port}",
                            timeout=datetime.timedelta(minutes=30), pg_options=streams.tp_group_options(backend))
    cpu = dist.new_group(backend="gloo", timeout=LONG)
    return dist.group.WORLD, cpu


def build_engine_on_group(cfg: EngineConfig, tp_pg, cpu_group, rank: int, world: int,
                          warmup: bool = True) -> ReplicatedEngine:
    """This rank's engine shard over existing process groups (`tp_pg`: the
    device collectives, RCCL on GPUs; `cpu_group`: gloo, event plane and
    setup exchanges) -- a TP group of its own (`build_tp_engine`) or a
    sub-group of a larger world (the disaggregated bench's engines)."""
    dev = torch.device(cfg.device)
    mc = get_config(cfg.model)
    custom = None
    if dev.type == "cuda" and world > 1:
        from . import custom_ar

        if custom_ar.enabled():  # one-shot xGMI all-reduce / all-gather for decode-size messages
            # None when the group's ranks share one device (custom_ar module docstring)
            custom = custom_ar.CustomAllReduce.create(cpu_group, rank, world, dev)
        if custom is None and cfg.use_cuda_graph and dist.get_backend(tp_pg) != "nccl":
            # a host-staged (gloo) TP collective cannot sit inside a hipGraph
            log.warning("TP rank %d: no custom all-reduce on a %s group -- decode graphs off", rank,
                        dist.get_backend(tp_pg))
            cfg.use_cuda_graph = False
    model = LlamaForCausalLM(mc, device=dev, tp=TPGroup(tp_pg, rank, world, custom_ar=custom))
    if not cfg.random_init and os.path.isdir(cfg.model):
        model.load_safetensors(cfg.model)
    elif world > 1 and cfg.shard_consistent_init:
        model.load_shard_from(LlamaForCausalLM(mc, device=dev).random_init(cfg.seed))
    else:
        model.random_init(cfg.seed)
    if cfg.quantization == "fp8":
        model.quantize_fp8()
    eng = LLMEngine(cfg, model_cfg=mc, model=model)
    if dev.type == "cuda" and warmup:
        # prefill GEMM kernels at the scheduler's chunk sizes, decode graphs
        # (every rank in lockstep: graph warm-up runs the TP collectives)
        eng.warmup()
    return ReplicatedEngine(eng, cpu_group, rank, world)


def build_tp_engine(cfg: EngineConfig, rank: int, world: int, master: str = "127.0.0.1", port: int = 29555,
                    base_gpu: int = 0, setup=None) -> ReplicatedEngine:
    """Build this rank's engine shard.  `setup` = (module, function, kwargs):
    function(rep, **kwargs) runs on the rank once the engine exists (followers
    use it to create their per-rank KV transfer endpoint)."""
    if cfg.device.startswith("cuda"):
        # DX_TP_SAME_GPU=1 (with DX_TP_BACKEND=gloo): every rank on base_gpu,
        # the functional GPU test of the TP engine on a one-GPU box
        gpu = base_gpu + (0 if os.environ.get("DX_TP_SAME_GPU") == "1" else rank)
        torch.cuda.set_device(gpu)
        cfg.device = f"cuda:{gpu}"
    dev = torch.device(cfg.device)
    tp_pg, cpu = init_tp_group(rank, world, master, port, dev)
    rep = build_engine_on_group(cfg, tp_pg, cpu, rank, world)
    if setup is not None:
        import importlib

        mod, fn, kw = setup
        getattr(importlib.import_module(mod), fn)(rep, **kw)
    return rep


def _follower_main(cfg_dict, rank, world, master, port, base_gpu, setup):
    cfg = EngineConfig(**cfg_dict)
    rep = build_tp_engine(cfg, rank, world, master, port, base_gpu, setup)
    rep.follower_loop()


def spawn_tp_engine(cfg: EngineConfig, tp: int, base_gpu: int = 0, port: int | None = None,
                    follower_setup=None) -> ReplicatedEngine:
    """Spawn TP followers (ranks 1..tp-1, one process per GPU) and return the
    rank-0 leader.  tp == 1 gives a single-process driver with the same API."""
    import dataclasses
    import multiprocessing as mp
    import socket

    if tp <= 1:
        if cfg.device.startswith("cuda"):
            torch.cuda.set_device(torch.device(cfg.device))
        return ReplicatedEngine(LLMEngine(cfg), None, 0, 1)
    if port is None:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    ctx = mp.get_context("spawn")
    procs = []
    for r in range(1, tp):
        p = ctx.Process(target=_follower_main,
                        args=(dataclasses.asdict(cfg), r, tp, "127.0.0.1", port, base_gpu, follower_setup),
                        daemon=True)
        p.start()
        procs.append(p)
    rep = build_tp_engine(cfg, 0, tp, "127.0.0.1", port, base_gpu)
    rep.followers = procs
    return rep


def make_tp_engine(cfg: EngineConfig, tp: int, base_gpu: int = 0, port: int | None = None):
    """Spawn TP followers and return a NativeEngine (token-level ABI) on rank 0."""
    from ..engine.engine import AsyncLLMEngine
    from ..llm.engines import NativeEngine

    rep = spawn_tp_engine(cfg, tp, base_gpu, port)
    ae = AsyncLLMEngine(rep).start()
    ne = NativeEngine(ae, rep.engine.eos_token_ids)
    ne.followers = rep.followers
    return ne
