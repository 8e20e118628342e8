"""Worker cores used by serving graphs and the `run` CLI.

* `LLMWorker` -- aggregated or decode worker (reference
  examples/llm/components/worker.py:50-229): native engine, KV event + load
  metrics publishers (worker id = lease id), and with `remote_prefill` the
  conditional-disaggregation decision per request (prefix hit, prefill queue
  depth, live thresholds), enqueueing RemotePrefillRequests and receiving the
  KV through the KVTransferAgent.
* `PrefillWorker` -- pulls the prefill queue, prefills (max_tokens = 1), ships
  KV + first token to the owning decode worker; drains and exits when its
  lease is revoked (prefill_worker.py:118-194).

Both drive a `ReplicatedEngine` leader (parallel/tp.py): with
`--tensor-parallel-size N` the worker spawns N-1 follower processes (one per
GPU of its allocation), each with its own KV transfer endpoint, and the KV
transfer runs per TP rank in lockstep (disagg/agent.py).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import time
import uuid

import torch

from ..disagg.agent import (_CP, KVTransferAgent, decode_leader_hook, install_decode, install_prefill,
                            prefill_leader_hook)
from ..disagg.prefill_queue import PrefillQueue, RemotePrefillRequest
from ..disagg.router import DisaggregatedRouter
from ..engine.engine import AsyncLLMEngine, EngineConfig
from ..engine.policy import PREFILL_ENGINE_DEFAULTS, SERVING_DEFAULTS
from ..parallel.tp import ReplicatedEngine, spawn_tp_engine
from ..engine.request import SamplingParams
from ..utils.faults import FAULTS
from .multimodal import decode_features, encode_urls, make_vision_encoder
from .kv_router import KvEventPublisher, KvMetricsPublisher

log = logging.getLogger("dynamo_exp_amd.workers")


def worker_arg_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--max-num-seqs", type=int, default=None,
                    help="request slots (default 256; prefill workers 32)")
    # scheduler defaults = engine/policy.py SERVING_DEFAULTS, what bench.py measures
    ap.add_argument("--max-num-batched-tokens", type=int, default=SERVING_DEFAULTS["max_num_batched_tokens"],
                    help="per-step token budget (prefill workers: at least 16384)")
    ap.add_argument("--gpu-memory-utilization", type=float, default=None,
                    help="fraction of device memory for weights + KV (default 0.9; prefill workers 0.5, raise it for "
                         "a TP1 prefill worker of a model that fills the GPU, e.g. 70B: the reference's 4P(TP1) "
                         "benchmark layout passes 0.9, examples/llm/benchmarks/disagg.yaml:45-56)")
    ap.add_argument("--num-gpu-blocks", type=int, default=None)
    ap.add_argument("--enable-prefix-caching", action="store_true", default=True)
    ap.add_argument("--remote-prefill", action="store_true")
    ap.add_argument("--conditional-disagg", action="store_true")
    # MI355X prefill saturation knee: the smallest ISL at which batch-1 prefill
    # reaches 85 % of its best rate (profiles/r4_prefill_curve.json: 89 % at 2000;
    # reference docs/guides/disagg_perf_tuning.md:60-70 derives it the same way)
    ap.add_argument("--max-local-prefill-length", type=int, default=2000)
    ap.add_argument("--max-prefill-queue-size", type=int, default=2)
    ap.add_argument("--router", default="round-robin")
    ap.add_argument("--tensor-parallel-size", type=int, default=1)
    ap.add_argument("--pipeline-parallel-size", type=int, default=1, help="only 1 is supported")
    ap.add_argument("--quantization", default=None, choices=[None, "fp8"])
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--device", default=None)
    ap.add_argument("--prefill-queue", default="prefill_queue")
    ap.add_argument("--min-read-tokens", type=int, default=256,
                    help="prefill worker: pull a decode worker's cached prompt prefix when it is at least this long "
                         "(shorter ones are recomputed)")
    ap.add_argument("--kv-transport", default="rccl", choices=["rccl", "host", "ipc"],
                    help="P->D KV bytes: rccl = device buffers over per-pair RCCL (prefill and decode workers on "
                         "distinct GPUs); host = pinned-host staging over gloo (lets both share one GPU); "
                         "ipc = one-sided WRITE into the decode worker's KV blocks through an IPC mapping "
                         "(prefill TP 1; distinct GPUs or one shared GPU; prefix READ one-sided as well). "
                         "Both sides must agree; never chosen implicitly")
    ap.add_argument("--host-kv-blocks", type=int, default=0, help="pinned-host KV tier size in blocks (0 = off)")
    ap.add_argument("--no-chunked-prefill", action="store_true")
    ap.add_argument("--max-prefill-streak", type=int, default=SERVING_DEFAULTS["max_prefill_streak"])
    ap.add_argument("--min-prefill-tokens", type=int, default=SERVING_DEFAULTS["min_prefill_tokens"],
                    help="prefill batching: hold new prompts (while streams decode) until this many tokens queue ...")
    ap.add_argument("--max-prefill-delay", type=float, default=SERVING_DEFAULTS["max_prefill_delay"],
                    help="... or the oldest has waited this long (s)")
    ap.add_argument("--prefill-hold-min-decode", type=int, default=SERVING_DEFAULTS["prefill_hold_min_decode"],
                    help="... and only while at least this many streams decode (light load: no hold)")
    ap.add_argument("--prefill-hold-partial", type=int, default=SERVING_DEFAULTS["prefill_hold_partial"],
                    help="while >= N streams decode, the hold also covers a split prompt's remainder (0 = off)")
    ap.add_argument("--prefill-whole-prompts", type=int, default=int(SERVING_DEFAULTS["prefill_whole_prompts"]))
    ap.add_argument("--engine", default="native", choices=["native", "sim"],
                    help="sim: the timing model of Llama-3-8B TP1 on one MI355X (engine/sim.py, no GPU) -- "
                         "serving-stack and planner studies on CPU")
    ap.add_argument("--sim-step-ms", type=float, default=0.0,
                    help="engine sim: fixed decode step time (0 = the calibrated MI355X model); serving-stack "
                         "load tests pin the per-stream token rate with it")
    ap.add_argument("--sim-slowdown", type=float, default=1.0,
                    help="engine sim: a virtual GPU k times slower than the MI355X model (step times x k, prefill "
                         "rate / k) -- planner studies in the overload regime of slower GPUs")
    ap.add_argument("--sim-gpu-gb", type=float, default=288.0,
                    help="engine sim: device memory of the virtual GPU (sizes the KV pool; e.g. 80 for an H100)")
    ap.add_argument("--metrics-port", type=int, default=0,
                    help="serve this worker's engine histograms (phases, KV transfer) on :PORT/metrics (0 = off; "
                         "deploy/metrics/prometheus.yml scrapes 9100+)")
    ap.add_argument("--encode-worker", default=None,
                    help="component serving `encode` for image inputs (multimodal); default: encode in-process")
    return ap


def parse_worker_args(argv: list[str]):
    a, _ = worker_arg_parser().parse_known_args(argv)
    from ..cli.run import check_pipeline_parallel

    check_pipeline_parallel(a.pipeline_parallel_size)
    return a


# role defaults for the flags a worker may leave unset: prefill engines run
# whole-prompt steps over few requests and share their GPU budget less
ROLE_DEFAULTS = {"prefill": {"max_num_seqs": 32, "gpu_memory_utilization": 0.5},
                 "decode": {"max_num_seqs": 256, "gpu_memory_utilization": 0.9}}


def role_value(a, name: str, prefill_only: bool):
    """A worker flag, or its role default when the flag was not given."""
    v = getattr(a, name, None)
    return ROLE_DEFAULTS["prefill" if prefill_only else "decode"][name] if v is None else v


def _engine(a, prefill_only: bool = False, follower_setup=None) -> ReplicatedEngine:
    max_seqs = role_value(a, "max_num_seqs", prefill_only)
    mem = role_value(a, "gpu_memory_utilization", prefill_only)
    if getattr(a, "engine", "native") == "sim":
        from ..engine.sim import SimLLMEngine

        kw = dict(max_num_seqs=max_seqs,
                  slowdown=getattr(a, "sim_slowdown", 1.0) or 1.0, gpu_gb=getattr(a, "sim_gpu_gb", 288.0) or 288.0)
        if getattr(a, "sim_step_ms", 0):
            kw.update(decode_ms=a.sim_step_ms, decode_per_seq_ms=0.0)
        return ReplicatedEngine(SimLLMEngine.mi355x_8b("prefill" if prefill_only else "decode", **kw), None, 0, 1)
    dev = a.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
    sched = dict(max_num_batched_tokens=a.max_num_batched_tokens,
                 max_prefill_streak=getattr(a, "max_prefill_streak", SERVING_DEFAULTS["max_prefill_streak"]),
                 chunked_prefill=not getattr(a, "no_chunked_prefill", False),
                 min_prefill_tokens=getattr(a, "min_prefill_tokens", 0),
                 max_prefill_delay=getattr(a, "max_prefill_delay", 0.0),
                 prefill_hold_min_decode=getattr(a, "prefill_hold_min_decode", 0),
                 prefill_hold_partial=getattr(a, "prefill_hold_partial", 0),
                 prefill_whole_prompts=bool(getattr(a, "prefill_whole_prompts", 0)))
    if prefill_only:  # bigger whole-prompt steps, never held (bench_disagg's prefill engines)
        sched.update(PREFILL_ENGINE_DEFAULTS,
                     max_num_batched_tokens=max(a.max_num_batched_tokens, PREFILL_ENGINE_DEFAULTS["max_num_batched_tokens"]))
    cfg = EngineConfig(model=a.model, block_size=a.block_size, max_model_len=a.max_model_len,
                       max_num_seqs=max_seqs, gpu_memory_utilization=mem,
                       num_gpu_blocks=a.num_gpu_blocks, use_cuda_graph=not (a.no_graph or prefill_only),
                       device=dev, host_kv_blocks=getattr(a, "host_kv_blocks", 0),
                       quantization=getattr(a, "quantization", None),
                       kv_cache_dtype=getattr(a, "kv_cache_dtype", "auto"),
                       # one-sided KV transport: prefill workers write into this cache
                       kv_shared=getattr(a, "kv_transport", None) == "ipc" and not prefill_only
                       and bool(getattr(a, "remote_prefill", False)), **sched)
    tp = max(1, int(getattr(a, "tensor_parallel_size", 1) or 1))
    rep = spawn_tp_engine(cfg, tp, follower_setup=follower_setup if tp > 1 else None)
    if tp == 1 and dev.startswith("cuda"):
        # prefill workers too: the GEMM kernels of the chunk sizes they run
        # load now, not as multi-second stalls of the first requests
        rep.engine.warmup()
    return rep


def _serve_engine_metrics(a, rep) -> None:
    port = int(getattr(a, "metrics_port", 0) or 0)
    if port:
        from prometheus_client import start_http_server

        start_http_server(port, registry=rep.engine.request_timer.registry)
        log.info("engine metrics on :%d/metrics", port)


def _follower_setup(role: str, drt, engine_id: str, ns: str, lease, kv_transport: str | None = None) -> tuple:
    return ("dynamo_exp_amd.disagg.agent", "follower_setup",
            dict(role=role, cp_address=drt.address, engine_id=engine_id, namespace=ns,
                 lease_id=lease.id if lease else None, kv_transport=kv_transport))


class LLMWorker:
    def __init__(self, args, drt, component, lease, namespace: str = "dynamo"):
        self.a, self.drt, self.component, self.lease = args, drt, component, lease
        self.ns = namespace
        self.engine: LLMEngine | None = None
        self.ae: AsyncLLMEngine | None = None
        self.agent: KVTransferAgent | None = None
        self.router = DisaggregatedRouter(args.max_local_prefill_length, args.max_prefill_queue_size,
                                          model=args.served_model_name or args.model,
                                          enabled=args.remote_prefill)
        self.queue = PrefillQueue(drt.cp, args.prefill_queue)
        self.engine_id = f"{lease.id:x}" if lease else uuid.uuid4().hex[:12]

    async def start(self) -> "LLMWorker":
        loop = self.loop = asyncio.get_running_loop()
        setup = _follower_setup("decode", self.drt, self.engine_id, self.ns, self.lease,
                                getattr(self.a, "kv_transport", None)) if self.a.remote_prefill else None
        self.engine = await asyncio.to_thread(_engine, self.a, False, setup)
        self.ae = AsyncLLMEngine(self.engine)
        _serve_engine_metrics(self.a, self.engine)
        wid = self.lease.id if self.lease else 0
        pub = KvEventPublisher(self.component, wid, self.a.block_size, loop)
        self.engine.add_kv_event_listener(pub.on_engine_events)
        self.metrics = await KvMetricsPublisher(self.component, wid, self.engine.forward_pass_metrics).start()
        if self.a.remote_prefill:
            rep = self.engine
            if getattr(self.a, "engine", "native") == "sim":
                from ..disagg.sim_agent import SimKVAgent, install_sim_decode

                self.agent = SimKVAgent(rep.engine, _CP(self.drt.cp, loop), self.engine_id, self.ns)
                await self.agent.start_async(self.drt.cp, self.lease.id if self.lease else None)
                self.ae.step_hooks.append(install_sim_decode(rep, self.agent))
            else:
                self.agent = KVTransferAgent(rep.engine, _CP(self.drt.cp, loop), self.engine_id, self.ns, 0,
                                             rep.world, kv_transport=getattr(self.a, "kv_transport", None))
                await self.agent.start_async(self.drt.cp, self.lease.id if self.lease else None)
                install_decode(rep, self.agent)
                self.ae.step_hooks.append(decode_leader_hook(rep, self.agent))
            self.engine.scheduler.on_remote_prefill = self._enqueue_remote
            await self.router.watch(self.drt.cp)
        self.ae.start()
        self._fault_task = FAULTS.start_lease_dropper(self.drt)
        return self

    def _enqueue_remote(self, req) -> None:
        """Engine thread: blocks are allocated; ask a prefill worker for the KV."""
        bs = self.engine.kv.block_size
        rp = RemotePrefillRequest(engine_id=self.engine_id, request_id=req.request_id, prompt_token_ids=req.prompt,
                                  block_ids=list(req.block_ids), skip_blocks=req.num_computed // bs,
                                  computed_block_ids=list(req.block_ids[: req.num_computed // bs]),
                                  engine_tp=self.engine.world)
        asyncio.run_coroutine_threadsafe(self.queue.enqueue(rp), self.loop)

    async def _image_embeds(self, urls: list[str]):
        """Image URLs -> ([n, hidden] embeddings, content hash): via the
        EncodeWorker component when configured, else an in-process encoder."""
        if getattr(self.a, "encode_worker", None):
            if getattr(self, "_enc_client", None) is None:
                comp = self.drt.namespace(self.ns).component(self.a.encode_worker)
                self._enc_client = await comp.endpoint("encode").client()
                await self._enc_client.wait_for_instances(timeout=120)
            out = None
            async for r in await self._enc_client.round_robin({"image_urls": urls}):
                out = r
            return decode_features(out, self.engine.model.device), out["hash"]
        if getattr(self, "_encoder", None) is None:
            self._encoder = await asyncio.to_thread(make_vision_encoder, self.engine.model_cfg, self.a.model,
                                                    str(self.engine.model.device))
        return await asyncio.to_thread(encode_urls, self._encoder, urls)

    async def generate(self, request: dict, ctx):
        FAULTS.on_request()
        mm = (request.get("multi_modal") or {}).get("image_urls")
        if mm:
            emb, h = await self._image_embeds(mm)
            params = SamplingParams.from_preprocessed(request, self.engine.eos_token_ids)
            rid = request.get("request_id") or ctx.id
            async for out in self.ae.generate(rid, request["token_ids"], params, context=ctx, mm_embeds=emb, mm_hash=h):
                yield out
            return
        remote = False
        if self.a.remote_prefill and not self.a.conditional_disagg:
            remote = True  # no disaggregated router: always prefill remotely (reference worker.py:185-196)
        elif self.a.remote_prefill:
            qsize = await self.queue.size()
            hit = (request.get("estimated_prefix_hit_num_blocks") or 0) * self.a.block_size
            remote = self.router.prefill_remote(len(request["token_ids"]), hit, qsize)
        params = SamplingParams.from_preprocessed(request, self.engine.eos_token_ids)
        rid = request.get("request_id") or ctx.id
        async for out in self.ae.generate(rid, request["token_ids"], params, remote_prefill=remote, context=ctx):
            yield out

    def stats(self) -> dict:
        return self.engine.forward_pass_metrics() if self.engine else {}

    def shutdown(self):
        if self.metrics:
            self.metrics.stop()
        if self.ae:
            self.ae.shutdown()
        _stop_followers(self.engine)


class PrefillWorker:
    def __init__(self, args, drt, component, lease, namespace: str = "dynamo"):
        self.a, self.drt, self.component, self.lease = args, drt, component, lease
        self.ns = namespace
        self.queue = PrefillQueue(drt.cp, args.prefill_queue)
        self.engine_id = f"p{lease.id:x}" if lease else uuid.uuid4().hex[:12]
        self.dequeued = 0
        self.busy = 0.0

    async def start(self) -> "PrefillWorker":
        loop = asyncio.get_running_loop()
        setup = _follower_setup("prefill", self.drt, self.engine_id, self.ns, self.lease,
                                getattr(self.a, "kv_transport", None))
        self.engine = await asyncio.to_thread(_engine, self.a, True, setup)
        rep = self.engine
        self.ae = AsyncLLMEngine(rep)
        _serve_engine_metrics(self.a, rep)
        if getattr(self.a, "engine", "native") == "sim":
            from ..disagg.sim_agent import SimKVAgent, install_sim_prefill

            self.agent = SimKVAgent(rep.engine, _CP(self.drt.cp, loop), self.engine_id, self.ns)
            await self.agent.start_async(self.drt.cp, self.lease.id if self.lease else None)
            self.ae.step_hooks.append(install_sim_prefill(rep, self.agent))
        else:
            self.agent = KVTransferAgent(rep.engine, _CP(self.drt.cp, loop), self.engine_id, self.ns, 0,
                                         rep.world, kv_transport=getattr(self.a, "kv_transport", None))
            await self.agent.start_async(self.drt.cp, self.lease.id if self.lease else None)
            install_prefill(rep, self.agent)
            self.ae.step_hooks.append(prefill_leader_hook(rep, self.agent))
        self.ae.start()
        self._busy_task = asyncio.create_task(self.track_busy())
        return self

    def device_seconds(self) -> float:
        """Engine device time so far: GPU time from the runner's per-launch
        events (native engine) or the timing model's device time (sim)."""
        eng = self.engine.engine
        runner = getattr(eng, "runner", None)
        if runner is not None:
            runner.harvest_gpu_time()
            return runner.timing["prefill_gpu"] + runner.timing["decode_gpu"]
        return float(getattr(eng, "timing", {}).get("device", 0.0))

    async def track_busy(self, period: float = 1.0) -> None:
        """`self.busy`: fraction of the last `period` seconds the engine's
        device was busy (the planner's prefill-utilization signal)."""
        t0, d0 = time.perf_counter(), self.device_seconds()
        while True:
            await asyncio.sleep(period)
            t1, d1 = time.perf_counter(), self.device_seconds()
            self.busy = min(1.0, max(0.0, (d1 - d0) / max(1e-6, t1 - t0)))
            t0, d0 = t1, d1

    @property
    def inflight(self) -> int:
        """Requests dequeued but not yet prefilled + shipped (two monotonic
        counters, each written by one thread)."""
        return self.dequeued - self.agent.stats["sent"]

    async def run(self) -> None:
        """Pull loop; stops pulling when the lease is revoked, then drains.
        Backpressure: a request is only pulled once the staging its KV
        transfer needs is reserved (agent.admit), so a slow decode side
        leaves work in the shared queue (where decode workers see the queue
        depth and prefill locally) instead of growing this worker's staging."""
        bs = self.a.block_size
        held = None  # a dequeued request waiting for staging
        while self.lease is None or self.lease.is_valid():
            if self.inflight >= 8:
                await asyncio.sleep(0.002)
                continue
            r = held or await self.queue.dequeue(timeout=1.0)
            held = None
            if r is None:
                continue
            if self.agent.is_cancelled(r.request_id):  # its decode worker prefilled it itself meanwhile
                continue
            # pull the decode worker's cached prefix instead of recomputing it
            # when it is long enough to be worth a round trip
            read = r.skip_blocks if r.skip_blocks * bs >= self.a.min_read_tokens else 0
            nblocks = (len(r.prompt_token_ids) + bs - 1) // bs - r.skip_blocks
            if r.engine_tp:
                self.agent.tp_cache[r.engine_id] = r.engine_tp
            ok = await asyncio.to_thread(self.agent.admit, r.request_id, nblocks, read, r.engine_id)
            if not ok:
                held = r
                await asyncio.sleep(0.002)
                continue
            self.dequeued += 1
            self.ae.call(self.engine.add_request, r.request_id, r.prompt_token_ids,
                         SamplingParams(max_tokens=1, ignore_eos=True), None, False, True,
                         self.agent.remote_meta(r, read))
        # drain: requests handed to the engine thread (ae.call) may not have
        # reached the engine yet -- count them through `inflight`, not only
        # through the engine's own queues
        while self.inflight > 0 or self.engine.has_unfinished() or self.agent.pending_sends():
            await asyncio.sleep(0.05)
        log.info("prefill worker %s drained", self.engine_id)

    def shutdown(self):
        t = getattr(self, "_busy_task", None)
        if t is not None:
            t.cancel()
        self.ae.shutdown()
        _stop_followers(self.engine)


def _stop_followers(rep) -> None:
    """Terminate TP follower processes (they block in the step broadcast)."""
    for p in getattr(rep, "followers", []) or []:
        if p.is_alive():
            p.terminate()
            p.join(5)
