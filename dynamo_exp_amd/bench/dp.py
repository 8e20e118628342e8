"""Aggregated data-parallel benchmark body (bench.py --gpus N --mode agg): the
same-node aggregated baseline the disaggregated layouts are compared with
("the 1/2/4/8-GPU scaling curve against an aggregated
single-engine baseline measured on the same node"; the reference's baseline
is two `vllm serve` TP4 engines behind nginx,
examples/llm/benchmarks/README.md:125-175).

N ranks form N / T aggregated engines of TP size T (`--tp`), each a
`ReplicatedEngine` over its own sub-groups (RCCL + the custom xGMI
all-reduce / all-gather, hipGraph decode).  Every engine leader runs its own
closed loop of `concurrency x T` streams (weak scaling: the per-GPU load is
fixed) or open loop, the timed windows are barrier-aligned across leaders,
then the fixed-QPS segment; the windows are merged like the disaggregated
bench's decode ranks.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

from ..engine.engine import EngineConfig
from ..parallel.tp import build_engine_on_group
from .serving import LoadGen, PromptGen, ServingWindow, closed_loop_request_rate, drive, fixed_qps_segment


def _log(rank, msg):
    if os.environ.get("DX_BENCH_VERBOSE") or rank == 0:
        print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)


def run_data_parallel(args, dev, rank: int, world: int):
    from ..disagg.bench_disagg import choose_transport

    transport = choose_transport(dev, world, getattr(args, "p2p_backend", "nccl"))
    backend = "nccl" if transport == "rccl" else "gloo"
    if not dist.is_initialized():
        dist.init_process_group(backend)
    one = torch.ones(1, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(one)
    comm_world = int(one.item())
    tp = max(1, int(getattr(args, "tp", 1) or 1))
    if world % tp:
        raise SystemExit(f"[bench] {world} GPUs do not divide into TP {tp} engines")
    cpu = dist.new_group(backend="gloo")
    mine = None
    for e in range(world // tp):
        rs = list(range(e * tp, (e + 1) * tp))
        tp_pg = dist.new_group(rs, backend=backend) if tp > 1 else None
        cg = dist.new_group(rs, backend="gloo") if tp > 1 else None
        if rank in rs:
            mine = (e, rs.index(rank), tp_pg, cg)
    leaders = dist.new_group(list(range(0, world, tp)), backend="gloo")
    eid, tp_rank, tp_pg, cg = mine
    conc = args.concurrency * tp
    cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=args.isl + args.osl + 64,
                       max_num_seqs=max(conc, 1) if args.qps is None else 256 * tp,
                       max_num_batched_tokens=args.max_batched_tokens, max_prefill_streak=args.max_prefill_streak,
                       use_cuda_graph=not args.no_graph, chunked_prefill=args.policy == "chunked", device=str(dev),
                       seed=args.seed, quantization=args.quantization,
                       kv_cache_dtype=getattr(args, "kv_cache_dtype", "auto"), min_prefill_tokens=args.min_prefill_tokens,
                       max_prefill_delay=args.max_prefill_delay, num_gpu_blocks=args.num_gpu_blocks,
                       prefill_hold_min_decode=args.prefill_hold_min_decode,
                       prefill_hold_partial=getattr(args, "prefill_hold_partial", 0),
                       prefill_whole_prompts=bool(getattr(args, "prefill_whole_prompts", 0)),
                       gpu_memory_utilization=args.gpu_mem_util or 0.90)
    gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 512)
          if s <= cfg.max_num_seqs]
    if cfg.max_num_seqs not in gs:
        gs.append(cfg.max_num_seqs)
    cfg.graph_sizes = tuple(gs)
    t0 = time.time()
    rep = build_engine_on_group(cfg, tp_pg, cg, tp_rank, tp, warmup=dev.type == "cuda")
    dist.barrier(group=cpu)
    _log(rank, f"agg engine {eid} (tp {tp_rank}/{tp}) ready in {time.time() - t0:.1f}s, "
               f"kv blocks {rep.engine.runner.num_blocks}")
    res = {"rank": rank, "leader": tp_rank == 0}
    if tp_rank == 0:
        eng = rep.engine
        win = ServingWindow()
        add = lambda rid, p, sp, cb: rep.add_request(rid, p, sp, on_output=cb)  # noqa: E731
        load = LoadGen(add, PromptGen(args.seed + 1000 * rank, args.isl, eng.model_cfg.vocab_size), args.osl, win,
                       rid_prefix=f"a{eid}-", seed=args.seed + rank)
        qps = args.qps * tp if args.qps is not None else None
        load.start_open(qps) if qps is not None else load.start_closed(conc)
        sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
        mix = drive(rep, load, win, args, sync, barrier=lambda: dist.barrier(group=leaders),
                    tag=f"a{eid} ", log=lambda m: _log(rank, m))
        load.stop()
        for rid in list(eng.requests):
            rep.abort(rid)
        qwin, qseg = None, 0.0
        if args.qps is None and args.qps_segment != 0:
            qseg = (args.qps_segment * tp) if args.qps_segment else 0.8 * closed_loop_request_rate(win, args.osl)
            dist.barrier(group=leaders)
            qwin = fixed_qps_segment(rep, add, PromptGen(args.seed + 7000 + rank, args.isl,
                                                         eng.model_cfg.vocab_size),
                                     args.osl, qseg, args.qps_seconds, sync=sync, rid_prefix=f"a{eid}-q",
                                     seed=args.seed + 13 * rank, log=lambda m: _log(rank, m))
            for rid in list(eng.requests):
                rep.abort(rid)
        while rep.has_unfinished():  # aborted requests leave the engine (followers apply the same events)
            rep.step()
        rep.shutdown()
        rep.step()
        res.update(window=win.state(), qps_window=qwin.state() if qwin is not None else None, qps=qseg,
                   engine_iters=mix["steps"], mixed_iters=mix["mixed_steps"], decode_iters=mix["decode_steps"])
    else:
        rep.follower_loop()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    rep.release()
    dist.barrier(group=cpu)
    gathered = [None] * world
    dist.all_gather_object(gathered, res, group=cpu)
    dist.barrier(group=cpu)
    dist.destroy_process_group()
    ls = [g for g in gathered if g["leader"]]
    win = ServingWindow.merged([g["window"] for g in ls])
    qs = [g["qps_window"] for g in ls if g.get("qps_window")]
    qwin = ServingWindow.merged(qs) if qs else None
    extra = {"parallelism": f"agg-dp{world // tp}-tp{tp}", "kv_transport": "none", "comm_world": comm_world,
             "engine_iters": sum(g.get("engine_iters", 0) for g in ls),
             "mixed_iters": sum(g.get("mixed_iters", 0) for g in ls)}
    if qwin is not None:
        extra["qps_segment"] = {"qps": round(sum(g.get("qps") or 0 for g in ls), 3), "seconds": args.qps_seconds}
    return win, extra, qwin
