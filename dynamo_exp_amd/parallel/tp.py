"""Tensor parallelism: one process per GPU, SPMD engines kept in lockstep.

Every TP rank runs a full LLMEngine over its weight shard (Megatron-style
column/row split, see models/llama.py) and the same deterministic scheduler /
block manager.  Only the leader (rank 0) receives requests; at the start of
each step it broadcasts the step's input *events* (new requests, aborts) over
a CPU (gloo) group, every rank applies them in the same order and steps.
Because sampling runs on all-gathered (bit-identical) logits with identical
seeds, all ranks pick the same tokens and their schedulers never diverge --
no per-step tensor broadcast of batch metadata is needed.  Activation
all-reduces go over RCCL (xGMI), captured inside the decode hipGraphs.

(The reference delegates TP to vLLM/SGLang: lib/engines/vllm0_8/src/lib.rs:371,
lib/engines/sglang/src/worker.rs:286-345.)
"""
from __future__ import annotations

import datetime
import logging
import os
import threading

import torch
import torch.distributed as dist

from ..engine.engine import EngineConfig, LLMEngine
from ..engine.request import SamplingParams
from ..models.config import get_config
from ..models.llama import LlamaForCausalLM, TPGroup

log = logging.getLogger("dynamo_exp_amd.tp")

LONG = datetime.timedelta(days=7)


class ReplicatedEngine:
    """Wraps an LLMEngine; rank 0 drives, followers mirror."""

    def __init__(self, engine: LLMEngine, cpu_group, rank: int):
        self.engine = engine
        self.group = cpu_group
        self.rank = rank
        self.pending: list[tuple] = []
        self._lock = threading.Lock()
        self.stopped = False

    # leader API (same signatures as LLMEngine)
    def add_request(self, request_id, prompt, params: SamplingParams, on_output=None, remote_prefill=False,
                    remote_decode=False, remote_meta=None):
        with self._lock:
            self.pending.append(("add", request_id, list(prompt), params, remote_prefill, remote_decode,
                                 remote_meta, on_output))

    def abort(self, request_id):
        with self._lock:
            self.pending.append(("abort", request_id))

    def shutdown(self):
        with self._lock:
            self.pending.append(("shutdown",))

    def has_unfinished(self) -> bool:
        return bool(self.pending) or self.engine.has_unfinished()

    def has_pending_work(self) -> bool:
        return bool(self.pending) or self.engine.scheduler.has_work()

    def __getattr__(self, name):
        return getattr(self.engine, name)

    def step(self):
        with self._lock:
            events, self.pending = self.pending, []
        callbacks = {}
        wire = []
        for e in events:
            if e[0] == "add":
                callbacks[e[1]] = e[7]
                wire.append(e[:7])
            else:
                wire.append(e)
        obj = [wire]
        dist.broadcast_object_list(obj, src=0, group=self.group)
        return self._apply_and_step(obj[0], callbacks)

    def _apply_and_step(self, events, callbacks):
        for e in events:
            if e[0] == "add":
                _, rid, prompt, params, rp, rd, meta = e
                self.engine.add_request(rid, prompt, params, callbacks.get(rid), rp, rd, meta)
            elif e[0] == "abort":
                self.engine.abort(e[1])
            elif e[0] == "shutdown":
                self.stopped = True
                return []
        return self.engine.step()

    def follower_loop(self) -> None:
        while not self.stopped:
            obj = [None]
            dist.broadcast_object_list(obj, src=0, group=self.group)
            self._apply_and_step(obj[0], {})


def init_tp_group(rank: int, world: int, master: str, port: int, device: torch.device):
    os.environ.setdefault("MASTER_ADDR", master)
    os.environ.setdefault("MASTER_PORT", str(port))
    backend = "nccl" if device.type == "cuda" else "gloo"
    dist.init_process_group(backend, rank=rank, world_size=world, init_method=f"tcp://{master}:{port}",
                            timeout=datetime.timedelta(minutes=30))
    cpu = dist.new_group(backend="gloo", timeout=LONG)
    return dist.group.WORLD, cpu


def build_tp_engine(cfg: EngineConfig, rank: int, world: int, master: str = "127.0.0.1", port: int = 29555,
                    base_gpu: int = 0) -> ReplicatedEngine:
    if cfg.device.startswith("cuda"):
        torch.cuda.set_device(base_gpu + rank)
        cfg.device = f"cuda:{base_gpu + rank}"
    dev = torch.device(cfg.device)
    tp_pg, cpu = init_tp_group(rank, world, master, port, dev)
    mc = get_config(cfg.model)
    custom = None
    if dev.type == "cuda" and world > 1:
        from . import custom_ar

        if custom_ar.enabled():  # one-shot xGMI all-reduce for decode-size messages
            custom = custom_ar.CustomAllReduce.create(cpu, rank, world, dev)
    model = LlamaForCausalLM(mc, device=dev, tp=TPGroup(tp_pg, rank, world, custom_ar=custom))
    model.random_init(cfg.seed) if cfg.random_init or not os.path.isdir(cfg.model) else model.load_safetensors(cfg.model)
    eng = LLMEngine(cfg, model_cfg=mc, model=model)
    if dev.type == "cuda":
        eng.warmup()
    return ReplicatedEngine(eng, cpu, rank)


def _follower_main(cfg_dict, rank, world, master, port, base_gpu):
    cfg = EngineConfig(**cfg_dict)
    rep = build_tp_engine(cfg, rank, world, master, port, base_gpu)
    rep.follower_loop()


def make_tp_engine(cfg: EngineConfig, tp: int, base_gpu: int = 0, port: int | None = None):
    """Spawn TP followers (ranks 1..tp-1) and return a NativeEngine on rank 0."""
    import dataclasses
    import multiprocessing as mp
    import socket

    from ..engine.engine import AsyncLLMEngine
    from ..llm.engines import NativeEngine

    if port is None:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    ctx = mp.get_context("spawn")
    procs = []
    for r in range(1, tp):
        p = ctx.Process(target=_follower_main, args=(dataclasses.asdict(cfg), r, tp, "127.0.0.1", port, base_gpu),
                        daemon=True)
        p.start()
        procs.append(p)
    rep = build_tp_engine(cfg, 0, tp, "127.0.0.1", port, base_gpu)
    ae = AsyncLLMEngine(rep).start()
    ne = NativeEngine(ae, rep.engine.eos_token_ids)
    ne.followers = procs
    return ne
