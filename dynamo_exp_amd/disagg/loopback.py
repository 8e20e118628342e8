"""1P1D in ONE process: a prefill engine and a decode engine on one device,
joined by the production KV transfer code (agent.KVTransferAgent +
transfer.KVDataPlane + the leader hooks the bench and the serving workers
install) over `transfer.LoopbackLinks` -- device-to-device copies with the
RCCL work contract -- and an in-process control plane.

What it is for: the device data plane (pack on the copy stream at each
layer-group boundary of the prefill forward, staging, matched send/recv,
unpack on the decode side, the prefix READ in the reverse direction) runs
exactly as on a multi-GPU node, with no host staging, on a box with ONE
GPU.  Only the wire (one hipMemcpyAsync on the hub's
stream instead of an RCCL kernel over xGMI) and the control plane (a dict
and a deque instead of dx-ctrld) differ.  The reference's counterpart is
the NIXL connector's asynchronous descriptor-list read / write
(container/deps/vllm/vllm_v0.8.4-dynamo-kv-disagg-patch.patch:1296-1424)
driven by its CopyStream (lib/llm/src/kv/layer.rs:785-1130).

With `kv_transport="ipc"` the same pair runs the one-sided WRITE instead
(prefill writes each layer group into the decode engine's blocks; no
staging, no receive side).

Used by tests/test_disagg_loopback.py (CPU and GPU) and
tools/loopback_disagg.py.
"""
from __future__ import annotations

import collections
import time

import msgpack

from ..engine.request import SamplingParams
from ..parallel.tp import ReplicatedEngine
from .agent import KVTransferAgent, decode_leader_hook, install_decode, install_prefill, prefill_leader_hook
from .prefill_queue import RemotePrefillRequest
from .router import DisaggregatedRouter
from .transfer import LoopbackHub, LoopbackLinks


class LoopbackControlPlane:
    """The agents' control-plane contract (`agent._CP`: blocking `call`,
    fire-and-forget `fire`) served from memory: transfer metadata in a dict,
    `publish` appends straight to the subscribed agent's inbox; a wire-subject
    message goes to every attached agent's wire filter, in publish order
    (the one ordered channel of agent.py's wire protocol)."""

    def __init__(self):
        self.kv: dict[str, bytes] = {}
        self.subs: dict[str, KVTransferAgent] = {}

    def attach(self, agent: KVTransferAgent) -> None:
        self.subs[agent.subject] = agent

    def call(self, name: str, *a, **kw):
        if name == "put":
            self.kv[a[0]] = a[1]
            return None
        if name == "get":
            return self.kv.get(a[0])
        raise ValueError(f"loopback control plane: no {name!r}")

    def fire(self, name: str, *a, **kw) -> None:
        if name != "publish":
            raise ValueError(f"loopback control plane: no {name!r}")
        if a[0].startswith("kv_wire."):
            m = msgpack.unpackb(a[1], raw=False)
            for agent in self.subs.values():
                if agent.wire_subject == a[0]:
                    agent._on_wire(m)
            return
        agent = self.subs.get(a[0])
        if agent is not None:
            agent.inbox.append(msgpack.unpackb(a[1], raw=False))


class Loopback1P1D:
    """Drive a prefill and a decode LLMEngine (same device) as one 1P1D
    deployment.  `add()` hands a request to the decode engine (the decode
    worker's role: it owns the request and allocates its blocks); with
    `remote=None` the conditional-disagg router decides (prompt longer than
    `max_local_prefill` and prefill queue shorter than `max_prefill_queue`).
    `step()` runs one iteration of both engine loops, in the order the bench's
    rank loops run them (disagg/bench_disagg.py _prefill_loop / _decode_loop)."""

    def __init__(self, prefill_engine, decode_engine, max_local_prefill: int = 0, max_prefill_queue: int = 1 << 30,
                 pool_cap_bytes: int | None = None, layer_group_count: int = 4, read_prefix: bool = True,
                 kv_transport: str | None = None):
        dev = decode_engine.runner.kv_cache.device
        self.hub = LoopbackHub(dev)
        self.cp = LoopbackControlPlane()
        self.p = ReplicatedEngine(prefill_engine, None, 0, 1)
        self.d = ReplicatedEngine(decode_engine, None, 0, 1)
        # kv_transport "ipc": the one-sided WRITE (the decode cache is in this process: written directly)
        mk = dict(namespace="loopback", pool_cap_bytes=pool_cap_bytes, layer_group_count=layer_group_count,
                  kv_transport=kv_transport)
        self.pa = KVTransferAgent(prefill_engine, self.cp, "p0", links=LoopbackLinks(self.hub, "p0"), **mk)
        self.da = KVTransferAgent(decode_engine, self.cp, "d0", links=LoopbackLinks(self.hub, "d0"), **mk)
        for a in (self.pa, self.da):
            a.start_sync()
            self.cp.attach(a)
        install_prefill(self.p, self.pa)
        install_decode(self.d, self.da)
        self.phook = prefill_leader_hook(self.p, self.pa)
        self.dhook = decode_leader_hook(self.d, self.da)
        self.router = DisaggregatedRouter(max_local_prefill, max_prefill_queue)
        self.read_prefix = read_prefix
        self.queue: collections.deque[RemotePrefillRequest] = collections.deque()
        self.bs = decode_engine.cfg.block_size
        decode_engine.scheduler.on_remote_prefill = self._on_remote
        self.counts = dict(remote=0, local=0, deferred=0)

    # decode worker: the request got its blocks -> prefill queue
    def _on_remote(self, req) -> None:
        self.queue.append(RemotePrefillRequest(engine_id=self.da.engine_id, request_id=req.request_id,
                                               prompt_token_ids=req.prompt, engine_tp=1,
                                               block_ids=list(req.block_ids),
                                               skip_blocks=req.num_computed // self.bs))

    def add(self, rid: str, prompt: list[int], params: SamplingParams, on_output=None, remote: bool | None = None):
        if remote is None:
            remote = self.router.prefill_remote(len(prompt), 0, len(self.queue))
        self.counts["remote" if remote else "local"] += 1
        self.d.add_request(rid, prompt, params, on_output=on_output, remote_prefill=remote)

    def _pull(self) -> None:
        """Prefill worker: dequeue while staging can be reserved."""
        while self.queue:
            r = self.queue[0]
            read = r.skip_blocks if self.read_prefix else 0
            nblocks = (len(r.prompt_token_ids) + self.bs - 1) // self.bs - r.skip_blocks
            if not self.pa.admit(r.request_id, nblocks, read, r.engine_id):
                self.counts["deferred"] += 1
                return
            self.queue.popleft()
            self.p.add_request(r.request_id, r.prompt_token_ids, SamplingParams(max_tokens=1, ignore_eos=True),
                               remote_decode=True,
                               remote_meta=self.pa.remote_meta(r, read))

    def step(self) -> None:
        self._pull()
        self.phook()
        if self.p.has_pending_work():
            self.p.step()
        self.dhook()
        if self.d.has_pending_work():
            self.d.step()

    def busy(self) -> bool:
        return bool(self.d.has_unfinished() or self.p.has_unfinished() or self.queue or self.pa.pending()
                    or self.da.pending() or self.dhook.pending() or self.pa.reservations)

    def run_until_idle(self, timeout: float = 600.0) -> None:
        t0 = time.time()
        while self.busy():
            self.step()
            if not (self.p.has_pending_work() or self.d.has_pending_work()):
                time.sleep(0.0002)  # transfers in flight on the device
            if time.time() - t0 > timeout:
                raise TimeoutError(f"loopback 1P1D not idle after {timeout}s: queue {len(self.queue)}, "
                                   f"prefill pending {self.pa.pending()}, decode pending {self.da.pending()}")
