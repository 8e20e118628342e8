"""Disaggregated xPyD serving benchmark body (bench.py, N > 1).

Ranks [0, x) are prefill workers, [x, N) decode workers (x = --prefill-ranks,
default N // 2).  Every decode rank owns `concurrency * N / y` in-flight
requests (closed loop) or `qps * N / y` requests/s (open loop), ISL/OSL fixed,
ignore_eos.  Admission applies conditional disaggregation
(:class:`DisaggregatedRouter`): long prompts go to the shared prefill queue
(control plane work queue) while it is short, else they are prefilled
locally.  Prefill ranks pull from the queue (token-budget bounded, so the
queue length seen by decode ranks stays honest), prefill in batches and
stream each request's KV blocks over xGMI in layer groups while the forward
pass is still running (RcclKVTransfer: announce before the forward, pack +
RCCL send per layer group on a copy stream, first token after it); the decode
rank posts the group receives on the announcement, unpacks into its
pre-allocated blocks and the request joins decode with its first token (TTFT
measured at the decode rank).  A prompt prefix the decode rank already caches
is pulled by the prefill rank (READ, reverse-direction process group) instead
of being recomputed.

Transport is explicit: RCCL device-to-device whenever the ranks run on GPUs,
unless `--p2p-backend gloo` asks for host staging (several ranks sharing one
GPU in functional tests).  A GPU run with fewer visible devices than ranks
and no such request exits with an error instead of silently measuring a
host-staged path.  The result reports `kv_transport` and `comm_world`, the
world size a device all-reduce of ones returned.
"""
from __future__ import annotations

import collections
import json
import os
import sys
import time

import msgpack
import torch
import torch.distributed as dist

from ..bench.serving import LoadGen, PromptGen, ServingWindow, drive
from ..engine.engine import EngineConfig, LLMEngine
from ..engine.request import SamplingParams
from ..runtime.control_plane import BackgroundServer, SyncControlPlaneClient
from .prefill_queue import PrefillQueue, RemotePrefillRequest
from .router import DisaggregatedRouter
from .transfer import RcclKVTransfer, init_pair_comms

QUEUE = "bench_prefill_queue"


def _log(rank, msg):
    if os.environ.get("DX_BENCH_VERBOSE") or rank == 0:
        print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def choose_transport(dev: torch.device, world: int, p2p_backend: str) -> str:
    """'rccl' (device buffers over RCCL), 'gloo-host' (GPU KV staged through
    host memory over gloo, only on request) or 'gloo' (CPU engines)."""
    if dev.type != "cuda":
        return "gloo"
    if p2p_backend == "gloo":
        return "gloo-host"
    n = torch.cuda.device_count()
    if n < world:
        raise SystemExit(f"[bench] {world} ranks but only {n} visible GPU(s): RCCL needs one GPU per rank; "
                         "pass --p2p-backend gloo to stage KV through host memory explicitly")
    return "rccl"


def start_control_plane():
    """Rank 0 hosts the bench's control plane (prefill queue, KV
    announcements, done flags).  The native epoll server (`dx-ctrld`) runs as
    a child process, so queue RPCs from every rank never wait on rank 0's
    GIL (its engine loop); the asyncio server on a thread is the fallback
    when the binary is not built.  Call before the process touches the GPU."""
    from ..runtime.control_plane import NativeServerProcess, use_native_server

    # ephemeral port: the address reaches the other ranks over the gloo group
    if use_native_server():
        return NativeServerProcess("0.0.0.0", 0, exit_with_parent=True).start()
    return BackgroundServer("0.0.0.0", 0).start()


def run_disaggregated(args, dev, rank: int, world: int, server=None):
    transport = choose_transport(dev, world, getattr(args, "p2p_backend", "nccl"))
    backend = "nccl" if transport == "rccl" else "gloo"
    if not dist.is_initialized():
        dist.init_process_group(backend)
    # one all-reduce of ones over the default (RCCL on GPUs) group: proves
    # every rank joined the device communicator
    one = torch.ones(1, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(one)
    comm_world = int(one.item())
    if comm_world != world:
        raise SystemExit(f"[bench] all-reduce world {comm_world} != WORLD_SIZE {world}")
    cpu = dist.new_group(backend="gloo")
    # decode -> prefill traffic (READ of cached prefixes) gets communicators of
    # its own: one in-order RCCL stream per direction and pair
    rev = dist.new_group(backend=backend)
    n_p = args.prefill_ranks if getattr(args, "prefill_ranks", None) else world // 2
    if not 0 < n_p < world:
        raise SystemExit(f"[bench] --prefill-ranks must be in [1, {world - 1}]")
    prefill_ranks = list(range(n_p))
    decode_ranks = list(range(n_p, world))
    is_prefill = rank in prefill_ranks
    d_group = dist.new_group(decode_ranks, backend="gloo")

    # ---- control plane (rank 0 hosts it)
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if rank == 0 and server is None:
        server = start_control_plane()
    port = [int(server.address.rsplit(":", 1)[1]) if rank == 0 else None]
    dist.broadcast_object_list(port, src=0, group=cpu)
    cp = SyncControlPlaneClient(f"{host}:{port[0]}")

    # ---- engines
    isl, osl = args.isl, args.osl
    max_len = isl + osl + 64
    nblk = getattr(args, "num_gpu_blocks", None)
    # weak scaling: the per-GPU load is fixed, so each decode rank owns
    # concurrency * world / n_decode in-flight requests (qps likewise)
    share = world / len(decode_ranks)
    conc = int(round(args.concurrency * share))
    qps = args.qps * share if getattr(args, "qps", None) else None
    max_seqs = conc if qps is None else 512
    if is_prefill:
        cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=max_len, max_num_seqs=32,
                           max_num_batched_tokens=max(args.max_batched_tokens, 16384), use_cuda_graph=False,
                           chunked_prefill=False, device=str(dev), seed=args.seed,
                           gpu_memory_utilization=getattr(args, "gpu_mem_util", None) or 0.5,
                           num_gpu_blocks=nblk, quantization=getattr(args, "quantization", None))
    else:
        cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=max_len,
                           max_num_seqs=max_seqs, max_num_batched_tokens=args.max_batched_tokens,
                           max_prefill_streak=args.max_prefill_streak, use_cuda_graph=not args.no_graph,
                           chunked_prefill=getattr(args, "policy", "chunked") == "chunked",
                           device=str(dev), seed=args.seed, num_gpu_blocks=nblk,
                           gpu_memory_utilization=getattr(args, "gpu_mem_util", None) or 0.9,
                           quantization=getattr(args, "quantization", None),
                           min_prefill_tokens=getattr(args, "min_prefill_tokens", 0),
                           max_prefill_delay=getattr(args, "max_prefill_delay", 0.0),
                           prefill_hold_min_decode=getattr(args, "prefill_hold_min_decode", 0))
    eng = LLMEngine(cfg)
    if dev.type == "cuda":
        if not is_prefill:
            gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 512)
                  if s <= max_seqs]
            if max_seqs not in gs:
                gs.append(max_seqs)
            eng.runner.cfg.graph_sizes = tuple(gs)
        eng.warmup()
    xfer = RcclKVTransfer(eng.runner.kv_cache, host_staging=transport == "gloo-host", rev_group=rev)
    init_pair_comms(rank, prefill_ranks, decode_ranks, dev if transport == "rccl" else "cpu", rev_group=rev)
    dist.barrier(group=cpu)
    _log(rank, f"{'prefill' if is_prefill else 'decode'} engine ready, kv blocks {eng.runner.num_blocks}, "
               f"transport {transport}")
    bs = args.block_size
    if is_prefill:
        res = _prefill_loop(args, rank, eng, xfer, cp, decode_ranks, bs)
    else:
        res = _decode_loop(args, rank, eng, xfer, cp, prefill_ranks, decode_ranks, bs, d_group, conc, qps)
    _sync(dev)
    dist.barrier(group=cpu)
    gathered = [None] * world
    dist.all_gather_object(gathered, res, group=cpu)
    cp.close()
    dist.barrier(group=cpu)
    if server is not None:
        server.stop()
    dist.destroy_process_group()
    win = ServingWindow.merged([g["window"] for g in gathered if g["role"] == "decode"])
    extra = {"parallelism": f"disagg-{n_p}P{world - n_p}D-tp1",
             "kv_transport": transport, "comm_world": comm_world,
             "engine_iters": sum(g.get("engine_iters", 0) for g in gathered),
             "remote_prefills": sum(g.get("remote", 0) for g in gathered),
             "local_prefills": sum(g.get("local", 0) for g in gathered),
             # bytes that crossed P->D, counted once (at the receiving decode ranks)
             "kv_transfer_GB": round(sum(g.get("xfer_bytes", 0) for g in gathered if g["role"] == "decode") / 1e9, 2),
             "kv_read_GB": round(sum(g.get("read_bytes", 0) for g in gathered if g["role"] == "decode") / 1e9, 2)}
    if rank == 0:
        _log(rank, "per-rank: " + json.dumps([{k: v for k, v in g.items() if k != "window"} for g in gathered]))
    return win, extra


def _prefill_loop(args, rank, eng, xfer, cp, decode_ranks, bs):
    pending_meta = {}

    def on_batch(batch):  # before the forward: announce the prompts it completes, one message per decode rank
        anns: dict[int, list] = {}
        for r, smp in zip(batch.requests[:batch.n_prefill], batch.sample):
            if smp and r.remote_decode:
                m = pending_meta[r.request_id]
                blocks = r.block_ids[m["skip"]:(len(r.prompt) + bs - 1) // bs]
                anns.setdefault(m["dst"], []).append(xfer.begin_send(r.request_id, blocks, m["dst"]))
        for dst, reqs in anns.items():
            cp.publish(f"bench.kv.{dst}", msgpack.packb({"t": "start", "src": rank, "reqs": reqs}))

    def on_prefilled(req):  # after the step: the first token
        m = pending_meta[req.request_id]
        cp.publish(f"bench.kv.{m['dst']}", msgpack.packb({"t": "done", "rid": req.request_id,
                                                           "tok": req.output[0], "lp": req.logprobs[0]}))

    def on_read(req, first, last):  # pull the decode rank's cached prefix blocks [first, last)
        m = pending_meta[req.request_id]
        cp.publish(f"bench.kv.{m['dst']}", msgpack.packb({"t": "read", "rid": req.request_id, "src": rank,
                                                           "first": first, "last": last}))
        xfer.post_read(req.request_id, m["dst"], req.block_ids[first:last])

    eng.batch_hook = on_batch
    eng.model.layer_hook = xfer.on_layer
    eng.prefill_done_hook = on_prefilled
    eng.scheduler.on_remote_read = on_read
    stopping = False
    sent = 0
    sends_done: set[str] = set()
    it = 0
    t_start = time.perf_counter()
    budget_tokens = eng.cfg.max_num_batched_tokens
    while True:
        it += 1
        if not stopping:
            budget = budget_tokens - sum(len(r.prompt) for r in eng.scheduler.waiting)
            while budget > 0:
                m = cp.q_pop(QUEUE, timeout=0.0 if eng.has_pending_work() else 0.002)
                if m is None:
                    break
                cp.q_ack(QUEUE, m["seq"])
                r = PrefillQueue.decode(m["data"])
                pending_meta[r.request_id] = {"dst": r.dst_rank, "skip": r.skip_blocks}
                eng.add_request(r.request_id, r.prompt_token_ids, SamplingParams(max_tokens=1, ignore_eos=True),
                                remote_decode=True, remote_read_blocks=r.skip_blocks)
                budget -= len(r.prompt_token_ids)
        if eng.has_pending_work():
            eng.step()
        xfer.end_forward()
        for rid in xfer.poll_reads():
            eng.finish_remote_read(rid)
        # a request's blocks are released once its sends completed AND its step was
        # applied (with asynchronous scheduling the sends can finish first)
        sends_done.update(xfer.poll_sends())
        for rid in [r for r in sends_done if r in eng.scheduler.transferring]:
            sends_done.discard(rid)
            eng.finish_transfer(rid)
            pending_meta.pop(rid, None)
            sent += 1
        if it % 4 == 0 or stopping:
            ndone = len(cp.get_prefix("bench/ddone/"))
            if ndone == len(decode_ranks):
                stopping = True
        if stopping and not eng.has_unfinished() and xfer.pending() == 0 and not sends_done:
            break
        if not eng.has_pending_work() and eng.scheduler.reading:
            time.sleep(0.0002)  # only waiting for pulled prefixes
    cp.put(f"bench/pdone/{rank}", b"1")
    return {"rank": rank, "role": "prefill", "sent": sent, "reads": xfer.stats["reads"],
            "xfer_bytes": xfer.stats["sent_bytes"], "busy_s": round(time.perf_counter() - t_start, 2),
            "prefill_tokens": eng.runner.timing["prefill_tokens"],
            "prefill_gpu_s": round(eng.runner.timing["prefill_gpu"], 2), "staging": dict(xfer.pool.stats)}


def _decode_loop(args, rank, eng, xfer, cp, prefill_ranks, decode_ranks, bs, d_group, conc, qps):
    max_q = args.max_prefill_queue if args.max_prefill_queue is not None else 4 * len(prefill_ranks)
    router = DisaggregatedRouter(args.max_local_prefill, max_q)
    inbox: collections.deque = collections.deque()
    cp.subscribe_callback(f"bench.kv.{rank}", lambda s, d: inbox.append(msgpack.unpackb(d, raw=False)))
    time.sleep(0.2)
    counts = dict(remote=0, local=0)
    queue_size = [0]
    tick = [0]

    def on_remote(req):
        rp = RemotePrefillRequest(engine_id=str(rank), request_id=req.request_id, prompt_token_ids=req.prompt,
                                  dst_rank=rank, skip_blocks=req.num_computed // bs)
        cp.q_push(QUEUE, PrefillQueue.encode(rp))
        queue_size[0] += 1

    eng.scheduler.on_remote_prefill = on_remote

    def add(rid, prompt, params, cb):
        remote = router.prefill_remote(len(prompt), 0, queue_size[0])
        counts["remote" if remote else "local"] += 1
        eng.add_request(rid, prompt, params, on_output=cb, remote_prefill=remote)

    def service():
        tick[0] += 1
        if tick[0] % 2 == 0:
            queue_size[0] = cp.q_size(QUEUE)
        while inbox:
            m = inbox.popleft()
            req = eng.scheduler.remote.get(m.get("rid"))
            if m["t"] == "start":  # post the layer-group receives (bytes of a cancelled request are dropped)
                items = []
                for a in m["reqs"]:
                    r = eng.scheduler.remote.get(a["rid"])
                    blocks = None
                    if r is not None:
                        skip = r.num_computed // bs
                        blocks = r.block_ids[skip:(len(r.prompt) + bs - 1) // bs]
                    items.append((a["rid"], a["nblocks"], blocks, a))
                xfer.post_recv_batch(m["src"], items)
            elif m["t"] == "done":
                xfer.sender_done(m["rid"], m)
            elif m["t"] == "read":  # serve our cached prefix blocks to the prefill rank
                n = m["last"] - m["first"]
                blocks = req.block_ids[m["first"]:m["last"]] if req is not None else [0] * n
                xfer.serve_read(m["rid"], blocks, m["src"])
        xfer.poll_served_reads()
        for rid, m in xfer.poll_recvs():
            if rid in eng.scheduler.remote:
                eng.finish_remote_prefill(rid, m["tok"], m["lp"])

    win = ServingWindow()
    load = LoadGen(add, PromptGen(args.seed + 1000 * rank, args.isl, eng.model_cfg.vocab_size), args.osl, win,
                   rid_prefix=f"d{rank}-", seed=args.seed + rank)
    if qps is not None:
        load.start_open(qps)
    else:
        load.start_closed(conc)
    dev = eng.model.device
    mix = drive(eng, load, win, args, lambda: _sync(dev), barrier=lambda: dist.barrier(group=d_group),
                service=service, tag=f"r{rank} ", log=lambda m: _log(rank, m))
    load.stop()
    cp.put(f"bench/ddone/{rank}", b"1")
    # drain: keep receiving until every prefill rank finished its sends
    while not (len(cp.get_prefix("bench/pdone/")) == len(prefill_ranks) and xfer.pending() == 0):
        service()
        time.sleep(0.0005)
    return {"rank": rank, "role": "decode", "window": win.state(), "engine_iters": mix["steps"],
            "mixed_iters": mix["mixed_steps"], "decode_iters": mix["decode_steps"],
            "remote": counts["remote"], "local": counts["local"], "xfer_bytes": xfer.stats["recv_bytes"],
            "read_bytes": xfer.stats["read_bytes"], "staging": dict(xfer.pool.stats),
            "decode_gpu_s": round(eng.runner.timing["decode_gpu"], 2),
            "prefill_gpu_s": round(eng.runner.timing["prefill_gpu"], 2)}
