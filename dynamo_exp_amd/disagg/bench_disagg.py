"""Disaggregated xPyD serving benchmark body (bench.py, N > 1).

Layout: the N ranks form prefill engines first, then decode engines; an
engine is a TP group of `--prefill-tp` / `--decode-tp` ranks (default `--tp`,
default 1).  `--prefill-ranks x` GPUs go to prefill (default N/2): x / ptp
prefill engines and (N - x) / dtp decode engines, e.g.

* `--gpus 8`                                   4P(tp1) + 4D(tp1)
* `--gpus 8 --tp 4 --model llama3-70b`         1P(tp4) + 1D(tp4) (BASELINE config 4)
* `--gpus 8 --prefill-tp 1 --decode-tp 4 --prefill-ranks 4`
                                               4P(tp1) + 1D(tp4), the reference's own
                                               single-node layout (examples/llm/benchmarks/
                                               disagg.yaml:45-56)

Every TP rank runs a `ReplicatedEngine` (parallel/tp.py) over its engine's
sub-groups: device collectives on RCCL (custom xGMI all-reduce / all-gather
for decode-size messages, captured in the decode hipGraphs), the event plane
on shared memory.  Engine leaders drive; followers mirror.

Each decode engine owns `concurrency * N / n_decode_engines` in-flight
requests (closed loop) or `qps * N / n_decode_engines` requests/s (open loop),
ISL/OSL fixed, ignore_eos.  Admission applies conditional disaggregation
(`DisaggregatedRouter`): long prompts go to the shared prefill queue (control
plane work queue) while it is short, else they are prefilled locally.
Prefill leaders pull the queue (token-budget and staging-reservation
bounded), prefill in batches and the KV moves over the ONE data plane the
serving graphs use (disagg/agent.py + transfer.KVDataPlane): layer-streamed
WRITE of each rank's relayout pieces over RCCL during the forward, READ of
prefixes the decode engine caches, staging backpressure.  Only the links
differ from serving: all ranks are one torch.distributed world here
(transfer.WorldLinks).  TTFT is measured at the decode leader.

Transport is explicit: RCCL device-to-device whenever the ranks run on GPUs,
unless `--p2p-backend gloo` asks for host staging (several ranks sharing one
GPU in functional tests).  A GPU run with fewer visible devices than ranks
and no such request exits with an error instead of silently measuring a
host-staged path.  The result reports `kv_transport`, `comm_world` (the
world size a device all-reduce of ones returned) and per-rank device-busy
time from CUDA events.
"""
from __future__ import annotations

import asyncio
import collections
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from ..bench.serving import LoadGen, PromptGen, ServingWindow, drive, fixed_qps_segment
from ..engine.engine import EngineConfig
from ..engine.request import SamplingParams
from ..parallel.tp import ReplicatedEngine, build_engine_on_group
from ..runtime.control_plane import BackgroundServer, SyncControlPlaneClient
from ..utils import streams
from .agent import (_CP, KVTransferAgent, decode_leader_hook, install_decode, install_prefill,
                    prefill_leader_hook)
from .prefill_queue import PrefillQueue, RemotePrefillRequest
from .router import DisaggregatedRouter
from .transfer import WorldLinks

QUEUE = "bench_prefill_queue"
NS = "bench"


def _log(rank, msg):
    if os.environ.get("DX_BENCH_VERBOSE") or rank == 0:
        print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def choose_transport(dev: torch.device, world: int, p2p_backend: str) -> str:
    """'rccl' (device buffers over RCCL), 'gloo-host' (GPU KV staged through
    host memory over gloo, only on request) or 'gloo' (CPU engines)."""
    if p2p_backend == "ipc":  # one-sided WRITE through the decode caches' mappings (any GPU count)
        return "ipc"
    if dev.type != "cuda":
        return "gloo"
    if p2p_backend == "gloo":
        return "gloo-host"
    n = torch.cuda.device_count()
    if n < world:
        raise SystemExit(f"[bench] {world} ranks but only {n} visible GPU(s): RCCL needs one GPU per rank; "
                         "pass --p2p-backend gloo to stage KV through host memory explicitly")
    return "rccl"


def plan_layout(world: int, prefill_ranks: int | None, ptp: int, dtp: int) -> tuple[dict, list, list]:
    """Engine ids -> global ranks: prefill engines p0.. on ranks [0, x), decode
    engines d0.. on [x, N).  Raises SystemExit on an impossible layout."""
    x = prefill_ranks if prefill_ranks else world // 2
    if not 0 < x < world:
        raise SystemExit(f"[bench] --prefill-ranks must be in [1, {world - 1}]")
    if x % ptp or (world - x) % dtp:
        raise SystemExit(f"[bench] {x} prefill GPUs / {world - x} decode GPUs do not divide into "
                         f"TP {ptp} prefill / TP {dtp} decode engines")
    ranks_of: dict[str, list[int]] = {}
    pre = [f"p{i}" for i in range(x // ptp)]
    dec = [f"d{j}" for j in range((world - x) // dtp)]
    for i, e in enumerate(pre):
        ranks_of[e] = list(range(i * ptp, (i + 1) * ptp))
    for j, e in enumerate(dec):
        ranks_of[e] = list(range(x + j * dtp, x + (j + 1) * dtp))
    return ranks_of, pre, dec


def parallelism_label(pre: list, dec: list, ptp: int, dtp: int) -> str:
    return f"disagg-{len(pre)}P(tp{ptp}){len(dec)}D(tp{dtp})"


def start_control_plane():
    """Rank 0 hosts the bench's control plane (prefill queue, KV
    notifications, transfer metadata, done flags).  The native epoll server
    (`dx-ctrld`) runs as a child process, so queue RPCs from every rank never
    wait on rank 0's GIL (its engine loop); the asyncio server on a thread is
    the fallback when the binary is not built.  Call before the process
    touches the GPU."""
    from ..runtime.control_plane import NativeServerProcess, use_native_server

    # ephemeral port: the address reaches the other ranks over the gloo group
    if use_native_server():
        return NativeServerProcess("0.0.0.0", 0, exit_with_parent=True).start()
    return BackgroundServer("0.0.0.0", 0).start()


def run_disaggregated(args, dev, rank: int, world: int, server=None):
    transport = choose_transport(dev, world, getattr(args, "p2p_backend", "nccl"))
    backend = "nccl" if transport == "rccl" else "gloo"
    if transport == "ipc" and dev.type == "cuda" and torch.cuda.device_count() >= world:
        backend = "nccl"  # TP collectives on RCCL; the KV bytes never touch it
    if not dist.is_initialized():
        dist.init_process_group(backend)
    # one all-reduce of ones over the default (RCCL on GPUs) group: proves
    # every rank joined the device communicator
    one = torch.ones(1, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(one)
    comm_world = int(one.item())
    if comm_world != world:
        raise SystemExit(f"[bench] all-reduce world {comm_world} != WORLD_SIZE {world}")
    ptp = getattr(args, "prefill_tp", None) or getattr(args, "tp", 1) or 1
    dtp = getattr(args, "decode_tp", None) or getattr(args, "tp", 1) or 1
    ranks_of, pre, dec = plan_layout(world, getattr(args, "prefill_ranks", None), ptp, dtp)

    # ---- groups (every rank creates every group, in one order)
    cpu = dist.new_group(backend="gloo")
    # decode -> prefill traffic (READ of cached prefixes) gets communicators of
    # its own: one in-order RCCL stream per direction and pair
    rev = dist.new_group(backend=backend)
    mine = None
    for e in pre + dec:
        rs = ranks_of[e]
        # TP collectives: high-priority RCCL streams (utils/streams.py); the KV p2p traffic stays normal
        tp_pg = dist.new_group(rs, backend=backend, pg_options=streams.tp_group_options(backend)) \
            if len(rs) > 1 else None
        cg = dist.new_group(rs, backend="gloo") if len(rs) > 1 else None
        if rank in rs:
            mine = (e, rs.index(rank), len(rs), tp_pg, cg)
    leaders = [ranks_of[e][0] for e in dec]
    d_group = dist.new_group(leaders, backend="gloo")
    engine_id, tp_rank, tp, tp_pg, cg = mine
    is_prefill = engine_id in pre
    leader = tp_rank == 0

    # ---- control plane (rank 0 hosts it)
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if rank == 0 and server is None:
        server = start_control_plane()
    port = [int(server.address.rsplit(":", 1)[1]) if rank == 0 else None]
    dist.broadcast_object_list(port, src=0, group=cpu)
    sc = SyncControlPlaneClient(f"{host}:{port[0]}")

    # ---- engines
    isl, osl = args.isl, args.osl
    max_len = isl + osl + 64
    nblk = getattr(args, "num_gpu_blocks", None)
    # weak scaling: the per-GPU load is fixed, so each decode engine owns
    # concurrency * world / n_decode_engines in-flight requests (qps likewise)
    share = world / len(dec)
    sweep = sweep_points(args)
    conc = int(round((max(sweep) if sweep else args.concurrency) * share))
    qps = args.qps * share if getattr(args, "qps", None) else None
    max_seqs = conc if qps is None else 512
    quant = getattr(args, "quantization", None)
    if is_prefill:
        # prefill ranks are sized by their own flags (role defaults 32 slots, 0.5 of the device)
        cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=max_len,
                           max_num_seqs=getattr(args, "prefill_max_seqs", None) or 32,
                           max_num_batched_tokens=max(args.max_batched_tokens, 16384), use_cuda_graph=False,
                           chunked_prefill=False, device=str(dev), seed=args.seed,
                           gpu_memory_utilization=getattr(args, "prefill_gpu_mem_util", None) or 0.5,
                           num_gpu_blocks=nblk, quantization=quant,
                           kv_cache_dtype=getattr(args, "kv_cache_dtype", "auto"))
    else:
        cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=max_len,
                           max_num_seqs=max_seqs, max_num_batched_tokens=args.max_batched_tokens,
                           max_prefill_streak=args.max_prefill_streak, use_cuda_graph=not args.no_graph,
                           chunked_prefill=getattr(args, "policy", "chunked") == "chunked",
                           device=str(dev), seed=args.seed, num_gpu_blocks=nblk,
                           gpu_memory_utilization=getattr(args, "gpu_mem_util", None) or 0.9,
                           quantization=quant, min_prefill_tokens=getattr(args, "min_prefill_tokens", 0),
                           kv_cache_dtype=getattr(args, "kv_cache_dtype", "auto"),
                           max_prefill_delay=getattr(args, "max_prefill_delay", 0.0),
                           prefill_hold_min_decode=getattr(args, "prefill_hold_min_decode", 0),
                           prefill_hold_partial=getattr(args, "prefill_hold_partial", 0),
                           prefill_whole_prompts=bool(getattr(args, "prefill_whole_prompts", 0)))
        gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 512)
              if s <= max_seqs]
        if max_seqs not in gs:
            gs.append(max_seqs)
        cfg.graph_sizes = tuple(gs)
    cfg.shard_consistent_init = bool(getattr(args, "verify_tokens", 0))
    # peers write into the decode caches (one-sided transport); on a GPU node the
    # RCCL runs share them too (measured free: profiles/r6_kvshared_ab.json), so
    # a failed RCCL preflight can fall back to the one-sided transport
    one_sided_ok = dev.type == "cuda" and ptp == 1
    cfg.kv_shared = not is_prefill and (transport == "ipc" or (transport in ("rccl", "gloo-host") and one_sided_ok))
    t0 = time.time()
    rep = build_engine_on_group(cfg, tp_pg, cg, tp_rank, tp, warmup=dev.type == "cuda")
    links = WorldLinks(ranks_of, group=dist.group.WORLD, rev_group=rev)
    agent = KVTransferAgent(rep.engine, _CP(sc.client, sc.loop), engine_id, NS, tp_rank, tp, links=links,
                            host_staging=transport == "gloo-host",
                            pool_cap_bytes=getattr(args, "staging_bytes", None),
                            kv_transport="ipc" if transport == "ipc" else None)
    if leader:
        asyncio.run_coroutine_threadsafe(agent.start_async(sc.client), sc.loop).result(30)
    else:
        agent.start_sync()
    if is_prefill:
        install_prefill(rep, agent)
    else:
        install_decode(rep, agent)
    fb = (transport in ("rccl", "gloo-host") and one_sided_ok
          and os.environ.get("DX_BENCH_IPC_FALLBACK", "1") != "0")
    warm_err = None
    if transport != "ipc":  # the one-sided WRITE uses no send / recv links
        try:
            links.warm(rank, pre, dec, dev if transport == "rccl" else "cpu")
        except Exception as e:  # noqa: BLE001 -- gathered below: every rank decides the same
            warm_err = repr(e)
    errs: list = [None] * world
    dist.all_gather_object(errs, warm_err, group=cpu)
    failed = [{"rank": r, "error": f"KV link warm-up: {e}"} for r, e in enumerate(errs) if e]
    if failed and not fb:
        _log(rank, "KV LINK WARM-UP FAILED: " + json.dumps(failed))
        raise SystemExit(3)
    dist.barrier(group=cpu)
    preflight = None
    if not failed and not getattr(args, "no_preflight", False):
        preflight = _preflight(rank, world, rep, agent, engine_id, is_prefill, ranks_of, pre, dec, dev, cpu,
                               fallback_ok=fb)
        if not preflight["ok"]:
            failed = preflight["failures"]
    if failed:  # every rank saw the same gathered verdict: all switch together
        _log(rank, "two-sided KV path failed -- switching to the one-sided transport: " + json.dumps(failed)[:2000])
        # abort the KV p2p communicators (ncclCommAbort): an RCCL kernel the
        # failed checks left waiting would otherwise hold its queue and hang
        # every device-wide synchronize after it
        for g in (dist.group.WORLD, rev):
            try:
                g._get_backend(dev).abort()
            except Exception as e:  # noqa: BLE001 -- best effort
                _log(rank, f"could not abort a KV communicator: {e!r}")
        old = agent
        for task in (getattr(old, "_sub_task", None), getattr(old, "_wire_task", None)):
            if task is not None:
                sc.loop.call_soon_threadsafe(task.cancel)
        agent = KVTransferAgent(rep.engine, _CP(sc.client, sc.loop), engine_id, NS, tp_rank, tp, links=links,
                                pool_cap_bytes=getattr(args, "staging_bytes", None), kv_transport="ipc")
        if leader:
            asyncio.run_coroutine_threadsafe(agent.start_async(sc.client), sc.loop).result(30)
        else:
            agent.start_sync()
        if is_prefill:
            install_prefill(rep, agent)
        else:
            install_decode(rep, agent)
        dist.barrier(group=cpu)
        preflight = _preflight(rank, world, rep, agent, engine_id, is_prefill, ranks_of, pre, dec, dev, cpu)
        preflight["fallback_from"] = {"transport": transport, "failures": failed}
        transport = "ipc"
    _log(rank, f"{engine_id} (tp {tp_rank}/{tp}) ready in {time.time() - t0:.1f}s, kv blocks "
               f"{rep.engine.runner.num_blocks}, transport {transport}")
    if not leader:
        t1, b0 = time.perf_counter(), _timing0(rep)
        rep.follower_loop()
        res = {"rank": rank, "role": "follower", "engine": engine_id, **_busy(rep, time.perf_counter() - t1, b0)}
    elif is_prefill:
        res = _prefill_loop(args, rank, rep, agent, sc, dec)
    else:
        res = _decode_loop(args, rank, rep, agent, sc, pre, dec, d_group, conc, qps, world_share=share)
    res["staging"] = dict(agent.pool.stats)
    res.update({k: agent.dp.stats[k] for k in ("sent_bytes", "recv_bytes", "read_bytes")})
    _sync(dev)
    rep.release()
    dist.barrier(group=cpu)
    gathered = [None] * world
    dist.all_gather_object(gathered, res, group=cpu)
    sc.close()
    dist.barrier(group=cpu)
    if server is not None:
        server.stop()
    dist.destroy_process_group()
    win = ServingWindow.merged([g["window"] for g in gathered if g["role"] == "decode"])
    if sweep:  # per concurrency point: every decode engine's window of that point, merged
        pts = []
        for i, c in enumerate(sweep):
            w = ServingWindow.merged([g["sweep"][i] for g in gathered if g["role"] == "decode"])
            sm = w.summary()
            itl = sm["itl_mean_ms"]
            pts.append({"concurrency_per_gpu": c, "tok_s_gpu": round(w.gen / w.elapsed / world, 1) if w.elapsed else 0.0,
                        "tok_s_user": round(1000.0 / itl, 2) if itl else None, **sm, "window_s": round(w.elapsed, 2)})
    qstates = [g["qps_window"] for g in gathered if g["role"] == "decode" and g.get("qps_window")]
    qwin = ServingWindow.merged(qstates) if qstates else None
    extra = {"parallelism": parallelism_label(pre, dec, ptp, dtp),
             "disagg_policy": disagg_policy(args, len(pre)),
             "preflight": preflight,
             "kv_transport": transport, "comm_world": comm_world,
             "prefill_engines": len(pre), "decode_engines": len(dec), "prefill_tp": ptp, "decode_tp": dtp,
             "engine_iters": sum(g.get("engine_iters", 0) for g in gathered),
             "remote_prefills": sum(g.get("remote", 0) for g in gathered),
             "local_prefills": sum(g.get("local", 0) for g in gathered),
             # bytes that crossed P->D (every decode rank receives its relayout pieces)
             # (one-sided: bytes the prefill ranks wrote into the decode caches)
             "kv_transfer_GB": round(sum(g.get("sent_bytes" if transport == "ipc" else "recv_bytes", 0)
                                         for g in gathered) / 1e9, 2),
             # prefix bytes served by decode ranks to prefill ranks (READ)
             "kv_read_GB": round(sum(g.get("read_bytes", 0) for g in gathered) / 1e9, 2),
             "staging_over_cap": sum(g["staging"].get("over_cap", 0) for g in gathered),
             # per remote request (decode leaders): prefill queue wait, forward start -> bytes landed,
             # landed -> decoding (ms)
             "transfer_spans": {g["engine"]: g.get("transfer_spans") for g in gathered
                                if g["role"] == "decode" and g.get("transfer_spans")},
             "staging_deferred": sum(g.get("deferred", 0) for g in gathered),
             "device_busy": {f"r{g['rank']}": g.get("busy_frac") for g in gathered}}
    vs = [g["verify"] for g in gathered if g.get("verify")]
    if vs:
        extra["verify"] = {k: sum(v.get(k, 0) for v in vs) for k in ("requests", "identical", "near_tie", "diverged")}
    if qwin is not None:
        extra["qps_segment"] = {"qps": round(sum(g.get("qps") or 0 for g in gathered), 3),
                                "seconds": args.qps_seconds}
    if sweep:
        extra["sweep_points"] = pts
    if rank == 0:
        _log(rank, "per-rank: " + json.dumps([{k: v for k, v in g.items() if k not in ("window", "qps_window", "sweep")}
                                              for g in gathered]))
    return win, extra, qwin


def sweep_points(args) -> list[int]:
    """--sweep c1,c2,...: closed-loop concurrencies PER GPU (the reference's
    genai-perf sweep, examples/llm/benchmarks/perf.sh:17-54), run one after
    the other on the same engines; [] = one closed-loop window."""
    sw = getattr(args, "sweep", None)
    return sorted({int(c) for c in sw.split(",") if c.strip()}) if sw else []


def disagg_policy(args, n_prefill_engines: int) -> dict:
    """What decides local vs remote prefill in this run (reported in the
    result's config).  `always`: every prompt goes to a prefill engine, the
    reference's benchmark setting (examples/llm/benchmarks/disagg.yaml:41-43,
    conditional-disagg: false); `conditional`: the reference's production
    DisaggregatedRouter rule (examples/llm/components/disagg_router.py:24-66)."""
    mode = getattr(args, "disagg_policy", "conditional")
    # each decode engine owns an equal closed loop (or Poisson stream): the
    # load split of the reference benchmark's round-robin router
    # (disagg.yaml:41-43); with distinct random prompts a KV-aware router has
    # no prefix to route on and reduces to the same balance
    router = "per-decode-engine load (round-robin equivalent)"
    if mode == "always":
        return {"mode": "always-remote", "router": router}
    q = args.max_prefill_queue if getattr(args, "max_prefill_queue", None) is not None else 4 * n_prefill_engines
    return {"mode": "conditional", "max_local_prefill": args.max_local_prefill, "max_prefill_queue": q,
            "router": router}


def _preflight(rank, world, rep, agent, engine_id, is_prefill, ranks_of, pre, dec, dev, cpu,
               fallback_ok: bool = False) -> dict:
    """Before any timed work: exact checks of this layout's TP collectives and
    of a WRITE + READ on every (prefill, decode) engine pair
    (disagg/preflight.py).  Gathered on every rank; any failure ends the run
    with exit status 3 -- a wrong cross-GPU path must not print a throughput.
    fallback_ok: a failure of the KV checks alone (TP collectives fine) is
    returned (ok False, "failures") for the caller to retry on the one-sided
    transport instead."""
    from .preflight import kv_check, kv_check_one_sided, tp_check

    t0 = time.perf_counter()
    mine = {"rank": rank, "engine": engine_id}
    try:
        # inference mode, as the engine's own steps: buffers the custom
        # all-reduce cached while the decode graphs were captured are
        # inference tensors, and writing them outside it raises
        with torch.inference_mode():
            mine["tp"] = tp_check(rep.engine.model.tp, dev)
            tps = {e: len(r) for e, r in ranks_of.items()}
            if agent.dp.one_sided:
                mine["kv"] = kv_check_one_sided(agent.dp, engine_id, is_prefill, pre, dec, tps,
                                                lambda: _active_barrier(cpu, dev))
            else:
                mine["kv"] = kv_check(agent.dp, engine_id, is_prefill, ranks_of, pre, dec, tps)
    except Exception as e:  # noqa: BLE001 -- reported below, on every rank
        mine["error"] = repr(e)
    for k in ("sent_bytes", "recv_bytes", "read_bytes", "sends", "recvs", "reads", "served"):
        agent.dp.stats[k] = 0  # the bench reports serving traffic only
    allv: list = [None] * world
    dist.all_gather_object(allv, mine, group=cpu)
    bad = [a for a in allv if a.get("error") or not a.get("tp", {}).get("ok") or not a.get("kv", {}).get("ok")]
    summary = {"ok": not bad, "seconds": round(time.perf_counter() - t0, 2),
               "tp_groups_checked": len({a["engine"] for a in allv if a.get("tp", {}).get("tp", 1) > 1}),
               "kv_pairs_checked": len(pre) * len(dec),
               "tp_paths": sorted({v["path"] for a in allv for k, v in a.get("tp", {}).items()
                                   if isinstance(v, dict) and "path" in v}),
               "graph_replay": all(a.get("tp", {}).get("graph_replay", True) for a in allv)}
    if bad and fallback_ok and all(a.get("tp", {}).get("ok") for a in allv):
        _log(rank, "KV PREFLIGHT FAILED: " + json.dumps(bad) + " -- retrying on the one-sided transport")
        summary["failures"] = bad
        return summary
    if bad:
        _log(rank, "PREFLIGHT FAILED: " + json.dumps(bad))
        if rank == 0:
            print(json.dumps({"preflight": summary, "failures": bad}), flush=True)
        raise SystemExit(3)
    _log(rank, f"preflight ok in {summary['seconds']}s: {summary}")
    return summary


def _active_barrier(group, dev, timeout: float = 300.0) -> None:
    """A barrier that keeps this process in HIP calls while it waits: a peer
    may be mapping this rank's KV cache (one-sided transport), and the import
    of an IPC handle completes only while the exporting process is inside the
    HIP runtime (profiles/r6_ipc_probe.json)."""
    w = dist.barrier(group=group, async_op=True)
    t0 = time.time()
    while not w.is_completed():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        time.sleep(0.001)
        if time.time() - t0 > timeout:
            raise RuntimeError(f"barrier not passed in {timeout}s")
    w.wait()


def _busy(rep, wall: float, base: dict | None = None) -> dict:
    """Device time from CUDA events (runner.timing *_gpu, minus the values at
    `base`, the start of this rank's serving loop) over the loop's wall time."""
    r = rep.engine.runner
    r.harvest_gpu_time()
    t = r.timing
    b = base or {}
    pg = t["prefill_gpu"] - b.get("prefill_gpu", 0.0)
    dg = t["decode_gpu"] - b.get("decode_gpu", 0.0)
    return {"prefill_gpu_s": round(pg, 2), "decode_gpu_s": round(dg, 2), "loop_s": round(wall, 2),
            "busy_frac": round((pg + dg) / wall, 3) if wall > 0 else None}


def _timing0(rep) -> dict:
    r = rep.engine.runner
    r.harvest_gpu_time()
    return dict(r.timing)


def _finish_engine(rep) -> None:
    """Leader: publish the shutdown event (followers leave follower_loop)."""
    rep.shutdown()
    rep.step()


def _prefill_loop(args, rank, rep, agent, sc, dec):
    hook = prefill_leader_hook(rep, agent)
    eng = rep.engine
    bs = args.block_size
    stopping = False
    held = None
    it = 0
    t_start, b0 = time.perf_counter(), _timing0(rep)
    budget_tokens = eng.cfg.max_num_batched_tokens
    prompt_tokens = 0
    beat = time.perf_counter()
    while True:
        it += 1
        if time.perf_counter() - beat > 30.0:  # progress line
            beat = time.perf_counter()
            _log(rank, f"prefill: {eng.stats['steps']} engine iterations, {prompt_tokens} prompt tokens, "
                       f"{len(agent.dp.sends)} sends in flight")
        if not stopping:
            budget = budget_tokens - sum(len(r.prompt) for r in eng.scheduler.waiting)
            while budget > 0:
                if held is None:
                    m = sc.q_pop(QUEUE, timeout=0.0 if rep.has_pending_work() else 0.002)
                    if m is None:
                        break
                    sc.q_ack(QUEUE, m["seq"])
                    held = PrefillQueue.decode(m["data"])
                    if agent.is_cancelled(held.request_id):  # its decode engine fell back meanwhile
                        held = None
                        continue
                r = held
                nblocks = (len(r.prompt_token_ids) + bs - 1) // bs - r.skip_blocks
                if r.engine_tp:
                    agent.tp_cache[r.engine_id] = r.engine_tp
                if not agent.admit(r.request_id, nblocks, r.skip_blocks, r.engine_id):
                    break  # staging full: the request waits here, the queue stays put
                held = None
                rep.add_request(r.request_id, r.prompt_token_ids, SamplingParams(max_tokens=1, ignore_eos=True),
                                remote_decode=True,
                                remote_meta=agent.remote_meta(r, r.skip_blocks))
                budget -= len(r.prompt_token_ids)
                prompt_tokens += len(r.prompt_token_ids)
        hook()
        if rep.has_pending_work():
            rep.step()
        elif rep.pending:
            rep.step()  # apply ext events (pulled prefixes landed)
        if it % 4 == 0 or stopping:
            if len(sc.get_prefix("bench/ddone/")) == len(dec):
                stopping = True
                held = None  # its decode engine aborted it
        if stopping and held is None and not rep.has_unfinished() and agent.dp.pending() == 0:
            break
        if not rep.has_pending_work() and (eng.scheduler.reading or agent.dp.sends):
            time.sleep(0.0002)  # waiting for pulled prefixes / sends to complete
            agent.dp.poll_sends()
    wall = time.perf_counter() - t_start
    _finish_engine(rep)
    sc.put(f"bench/pdone/{rank}", b"1")
    return {"rank": rank, "role": "prefill", "engine": agent.engine_id, "sent": agent.stats["sent"],
            "reads": agent.stats["reads"], "prefill_tokens": eng.runner.timing["prefill_tokens"], "prompt_tokens": prompt_tokens,
            "deferred": agent.stats["deferred"], **_busy(rep, wall, b0)}


def _segment_qps(args, win, share: float) -> float:
    from ..bench.serving import closed_loop_request_rate

    if getattr(args, "qps", None) is not None or getattr(args, "qps_segment", None) == 0:
        return 0.0
    if getattr(args, "qps_segment", None):
        return args.qps_segment * share
    return 0.8 * closed_loop_request_rate(win, args.osl)


def _verify_tokens(args, rank, rep, service) -> dict:
    """--verify-tokens K (default 2 for N > 1): K fixed prompts forced through
    the remote-prefill path of this layout -- prefill engine, relayout pieces
    over the links, decode engine -- must decode the greedy tokens that the
    SAME decode engine produces when it prefills those prompts itself (its
    prefix cache dropped in between, on every rank, so nothing transferred is
    reused).  Prefill and decode engines hold the same model
    (`shard_consistent_init` whenever verification is on), so this isolates
    the transfer.  No second model is built: it works for 70B TP4 decode
    engines as for 8B TP1.  A prefill engine of another TP size sums partial
    products in another order, so on random weights two near-tied logits can
    swap: a request whose first differing token has the same logprob in both
    runs (within 0.1 nats) is counted as a near-tie, not a transfer error."""
    eng = rep.engine
    k, n = args.verify_tokens, min(args.osl, 8)
    gen = PromptGen(args.seed + 99 + rank, args.isl, eng.model_cfg.vocab_size)
    prompts = [gen() for _ in range(k)]

    def run(tag: str, remote: bool) -> dict:
        outs: dict[str, list] = {}

        def cb(r, toks, lps, fin):
            outs.setdefault(r.request_id, []).extend(zip(toks, lps))

        for i, p in enumerate(prompts):
            rep.add_request(f"v{tag}{rank}-{i}", p, SamplingParams(max_tokens=n, ignore_eos=True), on_output=cb,
                            remote_prefill=remote)
        t0 = beat = time.time()
        while sum(len(v) == n for v in outs.values()) < k or rep.has_unfinished():
            service()
            if rep.has_pending_work():
                rep.step()
            else:
                time.sleep(0.0005)
            if time.time() - beat > 20.0:  # progress line (slow rehearsals on a shared GPU)
                beat = time.time()
                _log(rank, f"verify ({tag}): {sum(len(v) for v in outs.values())} tokens of {k * n}, "
                           f"{len(rep.engine.requests)} requests open, scheduler "
                           f"remote={len(rep.engine.scheduler.remote)} transferring={len(rep.engine.scheduler.transferring)}")
            if time.time() - t0 > 600:
                raise RuntimeError(f"verify: {'remote' if remote else 'local'} prefills did not complete")
        return {rid.split("-", 1)[1]: v for rid, v in outs.items()}

    def reset():  # every rank, lockstep: no transferred block may serve the local run as a prefix hit
        rep.submit("reset_prefix_cache", None)
        rep.step()

    got = run("r", True)
    reset()
    want = run("l", False)
    reset()
    same = near = 0
    for i, w in want.items():
        g = got[i]
        if [t for t, _ in g] == [t for t, _ in w]:
            same += 1
            continue
        j = next(x for x, (a, b) in enumerate(zip(g, w)) if a[0] != b[0])
        gap = abs(g[j][1] - w[j][1])
        near += gap < 0.1
        _log(rank, f"verify: prompt {i} differs from token {j} (logprob {g[j][1]:.3f} vs {w[j][1]:.3f})")
    _log(rank, f"verify: {same}/{k} remote-prefilled requests decode the local-prefill tokens, {near} near-tie swaps")
    return {"requests": k, "identical": same, "near_tie": near, "diverged": k - same - near}


def _decode_loop(args, rank, rep, agent, sc, pre, dec, d_group, conc, qps, world_share=1.0):
    eng = rep.engine
    bs = args.block_size
    n_pre = sum(1 for _ in pre)
    max_q = args.max_prefill_queue if args.max_prefill_queue is not None else 4 * n_pre
    always = getattr(args, "disagg_policy", "conditional") == "always"
    router = DisaggregatedRouter(0 if always else args.max_local_prefill, 1 << 30 if always else max_q)
    counts = dict(remote=0, local=0)
    queue_size = [0]
    tick = [0]
    hook = decode_leader_hook(rep, agent)
    agent.record_spans = True

    def on_remote(req):  # engine thread (leader): blocks allocated, ask a prefill engine for the KV
        agent.span(req.request_id, "enq")
        rp = RemotePrefillRequest(engine_id=agent.engine_id, request_id=req.request_id, prompt_token_ids=req.prompt,
                                  engine_tp=rep.world, skip_blocks=req.num_computed // bs,
                                  block_ids=list(req.block_ids))
        sc.q_push(QUEUE, PrefillQueue.encode(rp))
        queue_size[0] += 1

    eng.scheduler.on_remote_prefill = on_remote

    def add(rid, prompt, params, cb):
        remote = router.prefill_remote(len(prompt), 0, queue_size[0])
        counts["remote" if remote else "local"] += 1
        rep.add_request(rid, prompt, params, on_output=cb, remote_prefill=remote)

    def service():
        tick[0] += 1
        if tick[0] % 2 == 0:
            queue_size[0] = sc.q_size(QUEUE)
        hook()

    verify = _verify_tokens(args, rank, rep, service) if getattr(args, "verify_tokens", 0) else None
    dev = eng.model.device
    sweep_states = []
    for i, c in enumerate(sweep_points(args)):  # --sweep: one closed-loop window per point, same engines
        w = ServingWindow()
        ld = LoadGen(add, PromptGen(args.seed + 1000 * rank + 7 * i, args.isl, eng.model_cfg.vocab_size), args.osl, w,
                     rid_prefix=f"{agent.engine_id}-s{i}-", seed=args.seed + rank + 13 * i)
        ld.start_closed(max(1, int(round(c * world_share))))
        drive(rep, ld, w, args, lambda: _sync(dev), barrier=lambda: dist.barrier(group=d_group), service=service,
              tag=f"{agent.engine_id} C={c} ", log=lambda m: _log(rank, m))
        ld.stop()
        for rid in list(eng.requests):
            rep.abort(rid)
        sweep_states.append(w.state())
        _log(rank, f"sweep C={c}/GPU: {w.summary()}")
    win = ServingWindow()
    t_start, b0 = time.perf_counter(), _timing0(rep)
    mix = {"steps": 0, "mixed_steps": 0, "decode_steps": 0}
    if not sweep_states:  # the headline window (a sweep prints its points instead)
        load = LoadGen(add, PromptGen(args.seed + 1000 * rank, args.isl, eng.model_cfg.vocab_size), args.osl, win,
                       rid_prefix=f"{agent.engine_id}-", seed=args.seed + rank)
        if qps is not None:
            load.start_open(qps)
        else:
            load.start_closed(conc)
        mix = drive(rep, load, win, args, lambda: _sync(dev), barrier=lambda: dist.barrier(group=d_group),
                    service=service, tag=f"{agent.engine_id} ", log=lambda m: _log(rank, m))
        load.stop()
        for rid in list(eng.requests):  # the window is over: stop decoding, keep draining transfers
            rep.abort(rid)
    qwin = None
    qps_seg = 0.0 if sweep_states else _segment_qps(args, win, world_share)
    if qps_seg:  # fixed-QPS open-loop segment, same routing / disaggregation
        dist.barrier(group=d_group)
        qwin = fixed_qps_segment(rep, add, PromptGen(args.seed + 5000 + rank, args.isl, eng.model_cfg.vocab_size),
                                 args.osl, qps_seg, args.qps_seconds, service=service, sync=lambda: _sync(dev),
                                 rid_prefix=f"{agent.engine_id}-q", seed=args.seed + 31 * rank,
                                 log=lambda m: _log(rank, m))
        for rid in list(eng.requests):
            rep.abort(rid)
    sc.put(f"bench/ddone/{rank}", b"1")
    # drain: keep receiving (drop) until every prefill engine finished its sends
    while True:
        service()
        rep.step()
        if len(sc.get_prefix("bench/pdone/")) == n_pre and agent.pending() == 0 and not hook.pending() \
                and not rep.pending:
            break
        time.sleep(0.0005)
    wall = time.perf_counter() - t_start
    _finish_engine(rep)
    return {"rank": rank, "role": "decode", "engine": agent.engine_id, "window": win.state(), "sweep": sweep_states,
            "qps_window": qwin.state() if qwin is not None else None, "qps": qps_seg, "verify": verify,
            "engine_iters": mix["steps"], "mixed_iters": mix["mixed_steps"], "decode_iters": mix["decode_steps"],
            "remote": counts["remote"], "local": counts["local"], "deferred": agent.stats["deferred"],
            "transfer_spans": agent.span_summary(), **_busy(rep, wall, b0)}
