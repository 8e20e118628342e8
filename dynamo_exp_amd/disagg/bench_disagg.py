"""Disaggregated xPyD serving benchmark body (bench.py, N > 1).

Ranks [0, x) are prefill workers, [x, N) decode workers (x = N // 2).  Every
decode rank owns `concurrency` in-flight requests (closed loop, ISL/OSL fixed,
ignore_eos).  Admission applies conditional disaggregation
(:class:`DisaggregatedRouter`): long prompts go to the shared prefill queue
(control plane work queue) while it is short, else they are prefilled
locally.  Prefill ranks pull from the queue (token-budget bounded, so the
queue length seen by decode ranks stays honest), prefill in batches, and ship
each request's KV blocks with one RCCL send over xGMI; the decode rank
unpacks them into its pre-allocated blocks and the request joins decode with
its first token (TTFT measured at the decode rank).
"""
from __future__ import annotations

import collections
import json
import os
import sys
import threading
import time

import msgpack
import torch
import torch.distributed as dist

from ..engine.engine import EngineConfig, LLMEngine
from ..engine.request import SamplingParams
from ..runtime.control_plane import BackgroundServer, SyncControlPlaneClient
from .prefill_queue import PrefillQueue, RemotePrefillRequest
from .router import DisaggregatedRouter
from .transfer import RcclKVTransfer, init_pair_comms, transfer_bytes

QUEUE = "bench_prefill_queue"


def _log(rank, msg):
    if os.environ.get("DX_BENCH_VERBOSE") or rank == 0:
        print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run_disaggregated(args, dev, rank: int, world: int):
    # no device_id: keep lazily created per-pair p2p communicators (one RCCL
    # stream per prefill/decode pair -> no cross-pair ordering dependencies)
    # RCCL refuses two ranks of one communicator on the same device, so ranks
    # that share a GPU (world > visible devices) stage KV through host memory
    p2p_gloo = (dev.type != "cuda" or getattr(args, "p2p_backend", "nccl") == "gloo"
                or torch.cuda.device_count() < world)
    if not dist.is_initialized():
        dist.init_process_group("gloo" if p2p_gloo else "nccl")
    cpu = dist.new_group(backend="gloo")
    n_p = world // 2
    prefill_ranks = list(range(n_p))
    decode_ranks = list(range(n_p, world))
    is_prefill = rank in prefill_ranks
    d_group = dist.new_group(decode_ranks, backend="gloo")

    # ---- control plane (rank 0 hosts it)
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500")) + 17
    server = None
    if rank == 0:
        server = BackgroundServer("0.0.0.0", port).start()
    dist.barrier(group=cpu)
    cp = SyncControlPlaneClient(f"{host}:{port}")

    # ---- engines
    isl, osl = args.isl, args.osl
    max_len = isl + osl + 64
    nblk = getattr(args, "num_gpu_blocks", None)
    # weak scaling: `concurrency` is per GPU, so each decode rank owns
    # concurrency * world / n_decode in-flight requests
    conc = args.concurrency * world // len(decode_ranks)
    if is_prefill:
        cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=max_len, max_num_seqs=32,
                           max_num_batched_tokens=args.max_batched_tokens, use_cuda_graph=False, device=str(dev),
                           seed=args.seed, gpu_memory_utilization=getattr(args, "gpu_mem_util", None) or 0.5,
                           num_gpu_blocks=nblk, quantization=getattr(args, "quantization", None))
    else:
        cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=max_len,
                           max_num_seqs=conc, max_num_batched_tokens=args.max_batched_tokens,
                           max_prefill_streak=args.max_prefill_streak, use_cuda_graph=not args.no_graph,
                           chunked_prefill=getattr(args, "policy", "chunked") == "chunked",
                           device=str(dev), seed=args.seed, num_gpu_blocks=nblk,
                           gpu_memory_utilization=getattr(args, "gpu_mem_util", None) or 0.9,
                           quantization=getattr(args, "quantization", None),
                           min_prefill_tokens=getattr(args, "min_prefill_tokens", 0),
                           max_prefill_delay=getattr(args, "max_prefill_delay", 0.0))
    eng = LLMEngine(cfg)
    if not is_prefill:
        gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 512)
              if s <= conc]
        if conc not in gs:
            gs.append(conc)
        eng.runner.cfg.graph_sizes = tuple(gs)
        eng.warmup()
    host_staging = p2p_gloo and dev.type == "cuda"
    xfer = RcclKVTransfer(eng.runner.kv_cache, host_staging=host_staging)
    init_pair_comms(rank, prefill_ranks, decode_ranks, "cpu" if p2p_gloo else dev)
    dist.barrier(group=cpu)
    _log(rank, f"{'prefill' if is_prefill else 'decode'} engine ready, kv blocks {eng.runner.num_blocks}")
    bs = args.block_size
    if is_prefill:
        res = _prefill_loop(args, rank, eng, xfer, cp, decode_ranks, bs)
    else:
        res = _decode_loop(args, rank, eng, xfer, cp, prefill_ranks, decode_ranks, bs, d_group, conc)
    _sync(dev)
    dist.barrier(group=cpu)
    gathered = [None] * world
    dist.all_gather_object(gathered, res, group=cpu)
    cp.close()
    dist.barrier(group=cpu)
    if server is not None:
        server.stop()
    dist.destroy_process_group()
    gen = sum(g["gen"] for g in gathered)
    elapsed = max(g["elapsed"] for g in gathered)
    ttft = [t for g in gathered for t in g["ttft"]]
    extra = {"remote_prefills": sum(g.get("remote", 0) for g in gathered),
             "local_prefills": sum(g.get("local", 0) for g in gathered),
             "kv_transfer_GB": round(sum(g.get("xfer_bytes", 0) for g in gathered) / 1e9, 2)}
    if rank == 0:
        _log(rank, "per-rank: " + json.dumps([{k: v for k, v in g.items() if k != "ttft"} for g in gathered]))
    return gen, elapsed, ttft, extra


def _prefill_loop(args, rank, eng, xfer, cp, decode_ranks, bs):
    q = PrefillQueue(None, QUEUE)
    pending_meta = {}

    def on_prefilled(req):
        m = pending_meta[req.request_id]
        n_prompt_blocks = (len(req.prompt) + bs - 1) // bs
        blocks = req.block_ids[m["skip"]:n_prompt_blocks]
        nbytes = transfer_bytes(eng.runner.kv_cache, len(blocks))
        cp.publish(f"bench.kv.{m['dst']}", msgpack.packb({"rid": req.request_id, "src": rank, "nbytes": nbytes,
                                                           "tok": req.output[0], "lp": req.logprobs[0]}))
        xfer.send(req.request_id, blocks, m["dst"])

    eng.prefill_done_hook = on_prefilled
    stopping = False
    sent = 0
    it = 0
    t_start = time.perf_counter()
    while True:
        it += 1
        if not stopping:
            budget = args.max_batched_tokens - sum(len(r.prompt) for r in eng.scheduler.waiting)
            while budget > 0:
                m = cp.q_pop(QUEUE, timeout=0.0 if eng.scheduler.has_work() else 0.002)
                if m is None:
                    break
                cp.q_ack(QUEUE, m["seq"])
                r = PrefillQueue.decode(m["data"])
                pending_meta[r.request_id] = {"dst": r.dst_rank, "skip": r.skip_blocks}
                eng.add_request(r.request_id, r.prompt_token_ids,
                                SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True)
                budget -= len(r.prompt_token_ids)
        eng.step()
        for rid in xfer.poll_sends():
            eng.finish_transfer(rid)
            pending_meta.pop(rid, None)
            sent += 1
        if it % 4 == 0 or stopping:
            ndone = len(cp.get_prefix("bench/ddone/"))
            if ndone == len(decode_ranks):
                stopping = True
        if stopping and not eng.has_unfinished() and xfer.pending() == 0:
            break
    cp.put(f"bench/pdone/{rank}", b"1")
    return {"rank": rank, "role": "prefill", "gen": 0, "elapsed": 0.0, "ttft": [], "sent": sent,
            "xfer_bytes": xfer.stats["sent_bytes"], "busy_s": round(time.perf_counter() - t_start, 2),
            "prefill_tokens": eng.runner.timing["prefill_tokens"],
            "prefill_gpu_s": round(eng.runner.timing["prefill_gpu"], 2)}


def _decode_loop(args, rank, eng, xfer, cp, prefill_ranks, decode_ranks, bs, d_group, conc):
    import numpy as np

    rs = np.random.RandomState(args.seed + 1000 * rank)
    vocab = eng.model_cfg.vocab_size

    def gen_prompt():
        return rs.randint(min(1000, vocab // 4), vocab - min(1000, vocab // 4), size=args.isl).tolist()
    max_q = args.max_prefill_queue if args.max_prefill_queue is not None else 4 * len(prefill_ranks)
    router = DisaggregatedRouter(args.max_local_prefill, max_q)
    inbox: collections.deque = collections.deque()
    cp.subscribe_callback(f"bench.kv.{rank}", lambda s, d: inbox.append(msgpack.unpackb(d, raw=False)))
    time.sleep(0.2)
    state = dict(gen=0, ttft=[], counting=False, n=0, remote=0, local=0, admitting=True, fill=0)
    queue_size = [0]

    def on_remote(req):
        rp = RemotePrefillRequest(engine_id=str(rank), request_id=req.request_id, prompt_token_ids=req.prompt,
                                  dst_rank=rank, skip_blocks=req.num_computed // bs)
        cp.q_push(QUEUE, PrefillQueue.encode(rp))
        queue_size[0] += 1

    eng.scheduler.on_remote_prefill = on_remote

    def submit(osl=None):
        if not state["admitting"]:
            return
        state["n"] += 1
        rid = f"d{rank}-{state['n']}"
        osl = osl or args.osl
        params = SamplingParams(temperature=0.0, max_tokens=osl, min_tokens=osl, ignore_eos=True)
        arrival = time.perf_counter()
        prompt = gen_prompt()
        remote = router.prefill_remote(len(prompt), 0, queue_size[0])

        def on_output(req, toks, lps, fin, arrival=arrival):
            if state["counting"]:
                state["gen"] += len(toks)
                if req.first_token_time is not None and len(req.output) == len(toks) and toks:
                    state["ttft"].append(req.first_token_time - arrival)
            if fin:
                if osl != args.osl:
                    state["fill"] -= 1
                submit()

        if remote:
            state["remote"] += 1
        else:
            state["local"] += 1
        eng.add_request(rid, prompt, params, on_output=on_output, remote_prefill=remote)

    # steady-state fill (bench.py stagger_lengths): staggered initial output
    # lengths, run until every initial stream finished, then W + K steps
    fill = [max(1, (i + 1) * args.osl // conc) for i in range(conc)]
    state["fill"] = sum(1 for o in fill if o != args.osl)
    for o in fill:
        submit(o)

    def service():
        while inbox:
            m = inbox.popleft()
            req = eng.scheduler.remote.get(m["rid"])
            if req is None:
                continue
            skip = req.num_computed // bs
            n_prompt_blocks = (len(req.prompt) + bs - 1) // bs
            xfer.post_recv(m["rid"], m["src"], m["nbytes"], req.block_ids[skip:n_prompt_blocks], m)
        for rid, m in xfer.poll_recvs():
            eng.finish_remote_prefill(rid, m["tok"], m["lp"])

    fill_steps = 0
    while state["fill"] > 0:
        if fill_steps % 2 == 0:
            queue_size[0] = cp.q_size(QUEUE)
        service()
        if eng.scheduler.has_work():
            eng.step()
            fill_steps += 1
        else:
            time.sleep(0.0005)
    _log(rank, f"steady-state fill done after {fill_steps} steps")
    steps = 0
    t_start = t_end = None
    total = args.warmup + args.steps
    while True:
        if steps == args.warmup and t_start is None:
            _sync(eng.model.device)
            dist.barrier(group=d_group)
            t_start = time.perf_counter()
            state["counting"] = True
        if steps % 2 == 0:
            queue_size[0] = cp.q_size(QUEUE)
        service()
        if eng.scheduler.has_work():
            eng.step()
            steps += 1
        else:
            time.sleep(0.0005)
        if steps >= total and t_end is None:
            _sync(eng.model.device)
            t_end = time.perf_counter()
            state["counting"] = False
            state["admitting"] = False
            cp.put(f"bench/ddone/{rank}", b"1")
        if t_end is not None:
            # drain: keep receiving until every prefill rank finished its sends
            if len(cp.get_prefix("bench/pdone/")) == len(prefill_ranks) and xfer.pending() == 0:
                service()
                break
    return {"rank": rank, "role": "decode", "gen": state["gen"], "elapsed": t_end - t_start, "ttft": state["ttft"],
            "remote": state["remote"], "local": state["local"], "xfer_bytes": xfer.stats["recv_bytes"],
            "decode_gpu_s": round(eng.runner.timing["decode_gpu"], 2),
            "prefill_gpu_s": round(eng.runner.timing["prefill_gpu"], 2)}
