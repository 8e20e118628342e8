#!/usr/bin/env python3
"""Headline benchmark: Llama-3-8B serving throughput on MI355X.

Metric (BASELINE.json): output tokens/sec of the node + p50 TTFT, Llama-3-8B,
synthetic ISL 3000 / OSL 150 requests with ignore_eos (the reference's
genai-perf methodology, examples/llm/benchmarks/perf.sh:17-54).  Default:
closed loop at a fixed per-GPU concurrency (weak scaling: per-GPU load fixed
as N grows); `--qps R` runs open loop at R requests/s per GPU (Poisson
arrivals) and reports TTFT "at fixed QPS".

* N = 1: aggregated engine (prefill + decode on one GPU, TP1, bf16).
* N > 1: disaggregated xPyD (default x = y = N/2: 1P1D .. 4P4D), one rank per
  GPU over RCCL.  Each decode rank owns its requests; prompts longer than the
  conditional-disagg threshold are prefilled on a prefill rank and the KV
  blocks come back over RCCL (xGMI) send/recv; decode ranks prefill locally
  while the prefill queue is full (examples/llm/components/disagg_router.py:24-66).
  Launched by torchrun (RANK/WORLD_SIZE in the env), or `--gpus N` alone:
  bench.py then starts the N rank processes itself (the parent makes no GPU
  call) and exits with their status.

Timed window.  One bench step = `--iters-per-step` engine iterations of the
engine (N = 1) or of every decode rank (N > 1), by default OSL/5 = 30, so five
steps span one OSL cycle.  Why not one iteration: an iteration that carries
prompt chunks costs ~6x a decode-only one, and a closed loop with a fixed OSL
keeps a phase structure with period ~OSL iterations (requests admitted
together finish together and their replacements are admitted together again;
profiles/r2_bench_phase_trace.txt shows one slow block per 150 iterations).
A window of single iterations measured wherever it landed in that cycle
(BENCH_r01: 1600 tok/s over 20 iterations vs 3016 over 500); K steps that are
a multiple of 5 cover whole cycles whatever the starting phase.  W untimed
warmup steps after the steady-state fill (bench/serving.py), then exactly K
timed steps bracketed by barrier + synchronize; value = output tokens
generated inside the window over all ranks / max window over ranks.
Weights are random-init with the real architecture; data is synthetic.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from dynamo_exp_amd.engine.policy import SERVING_DEFAULTS as SD  # noqa: E402 -- torch-free

METRIC = "output tokens/sec (node) + p50 TTFT at fixed QPS"
MODEL_NAMES = {"llama3-8b": "Llama-3-8B", "llama3-70b": "Llama-3-70B",
               "deepseek-r1-distill-llama-8b": "DeepSeek-R1-Distill-Llama-8B"}


def metric_label(model: str, parallelism: str) -> str:
    """BASELINE.json's metric, labelled with what this run actually is: an
    aggregated run must not claim the disaggregated layout."""
    name = MODEL_NAMES.get(model, model)
    if parallelism.startswith("disagg-"):
        return f"{METRIC}, {name} {parallelism}"
    if parallelism == "agg-tp1":
        return f"{METRIC}, {name} aggregated ({parallelism}); BASELINE config 2"
    return f"{METRIC}, {name} aggregated data-parallel ({parallelism}); same-node baseline"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--iters-per-step", type=int, default=None,
                    help="engine iterations per bench step (decode-rank iterations for N > 1); default OSL/5, "
                         "so 5 steps span one OSL cycle")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--concurrency", type=int, default=128,
                    help="closed loop: in-flight requests per GPU (decode ranks own concurrency*N/n_decode each)")
    ap.add_argument("--qps", type=float, default=None,
                    help="open loop: Poisson arrivals at this many requests/s per GPU (TTFT at fixed QPS)")
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="per-step token budget (default 8192 chunked, 16384 prefill-first)")
    ap.add_argument("--policy", default="chunked", choices=["chunked", "prefill-first"],
                    help="chunked = mixed prefill-chunk + decode batches; prefill-first = whole-prompt prefill steps")
    # scheduler defaults: engine/policy.py SERVING_DEFAULTS, the same ones `run out=native`
    # and the graph workers serve with
    ap.add_argument("--max-prefill-streak", type=int, default=SD["max_prefill_streak"])
    ap.add_argument("--min-prefill-tokens", type=int, default=SD["min_prefill_tokens"],
                    help="prefill batching: while streams decode, hold new prompts until this many tokens are "
                         "queued ... (0 = off; profiles/r1_prefill_batching_sweep.json)")
    ap.add_argument("--max-prefill-delay", type=float, default=SD["max_prefill_delay"], help="... or the oldest waited this long (s)")
    ap.add_argument("--prefill-hold-min-decode", type=int, default=SD["prefill_hold_min_decode"],
                    help="... and only while at least this many streams decode (0 = always): the closed-loop "
                         "C=128 engine (~125 decoding) holds, the fixed-QPS point (~45) does not -- TTFT p50 "
                         "there 138 -> 100 ms at unchanged tok/s (profiles/r4_hold_min_decode_ab.txt; 48 in r2)")
    ap.add_argument("--prefill-hold-partial", type=int, default=SD["prefill_hold_partial"],
                    help="N > 0: while >= N streams decode, the hold also covers a prompt remainder split off "
                         "by the token budget -- every mixed step a full 8192-token step under saturation "
                         "(+1.7 %% tok/s, TTFT at fixed QPS unchanged; 0 = off; profiles/r4_prefill_hold_partial_ab.txt)")
    ap.add_argument("--prefill-whole-prompts", type=int, default=0,
                    help="1: past half the step budget, a new prompt that does not fit whole waits for the next "
                         "step instead of being split")
    ap.add_argument("--prefill-ranks", type=int, default=None,
                    help="N > 1: GPUs for prefill engines (default N/2); the rest run decode engines")
    ap.add_argument("--mode", default="disagg", choices=["disagg", "agg"],
                    help="N > 1: disagg = xPyD prefill/decode engines (default); agg = N/TP aggregated engines "
                         "(data parallel), the same-node aggregated baseline")
    ap.add_argument("--tp", type=int, default=1, help="N > 1: TP size of every engine (prefill and decode)")
    ap.add_argument("--prefill-tp", type=int, default=None, help="TP size of prefill engines (default --tp)")
    ap.add_argument("--decode-tp", type=int, default=None, help="TP size of decode engines (default --tp)")
    ap.add_argument("--staging-bytes", type=int, default=None,
                    help="KV transfer staging pool cap per rank (bytes; default 4 GiB): backpressure bound")
    ap.add_argument("--qps-segment", type=float, default=None,
                    help="after the closed-loop window: an open-loop Poisson segment at this many requests/s "
                         "per GPU (default 0.8 x the closed-loop request rate; 0 = skip) for TTFT at fixed QPS")
    ap.add_argument("--qps-seconds", type=float, default=12.0, help="measured length of the fixed-QPS segment")
    ap.add_argument("--verify-tokens", type=int, default=None,
                    help="N > 1 disagg: before the window, decode K fixed prompts through the remote-prefill path "
                         "and compare with the same decode engine prefilling them itself (config.verify; default 2, "
                         "0 = off)")
    ap.add_argument("--no-preflight", action="store_true",
                    help="N > 1 disagg: skip the exact TP-collective and KV WRITE/READ checks (config.preflight)")
    ap.add_argument("--disagg-policy", default="conditional", choices=["conditional", "always"],
                    help="N > 1 disagg: conditional = the DisaggregatedRouter rule (--max-local-prefill, "
                         "--max-prefill-queue); always = every prompt prefilled remotely (the reference's "
                         "benchmark setting, examples/llm/benchmarks/disagg.yaml:41-43)")
    ap.add_argument("--max-local-prefill", type=int, default=2000,
                    help="conditional disagg: prompts longer than this go to the prefill rank.  Rule: the smallest "
                         "ISL at which batch-1 prefill reaches 85 %% of its best rate -- the reference's saturation "
                         "point (docs/guides/disagg_perf_tuning.md:60-70) -- 2000 on MI355X "
                         "(profiles/r4_prefill_curve.json: 89 %% at 2000, 83 %% at 1500).  At that file's stricter "
                         "90 %% reading the knee is 3000, which would keep every ISL-3000 bench prompt local")
    ap.add_argument("--max-prefill-queue", type=int, default=None,
                    help="conditional disagg: remote only while the shared prefill queue is shorter than this "
                         "(default 4 per prefill rank)")
    ap.add_argument("--sweep", default=None,
                    help="closed-loop concurrency sweep, e.g. 1,2,4,8,16,32,64,128,256 (per GPU; N > 1: the xPyD "
                         "layout's decode engines, then the usual window) -- one engine, each "
                         "point a full fill + warmup + timed window; prints ONE JSON line with a point per "
                         "concurrency (tok/s/GPU vs tok/s/user, TTFT, ITL): the reference's comparison method "
                         "(examples/llm/benchmarks/perf.sh:17-54), not the driver's headline line")
    ap.add_argument("--remote-frac", type=float, default=0.0,
                    help="N = 1 --sweep study mode (tools/disagg_projection.py): each request is remotely "
                         "prefilled with this probability -- blocks allocated, KV taken as arrived -- so one GPU "
                         "measures the decode role of an xPyD layout whose decode engines prefill the other "
                         "1 - q of the prompts locally (1 = pure decode role)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gemm-report", default=None, help="write the decode-GEMM tuning table (JSON) here")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--trace-steps", action="store_true", help="log throughput of every bench step (stderr)")
    ap.add_argument("--cpu", action="store_true", help="CPU reference path (tests only)")
    ap.add_argument("--quantization", default=None, choices=[None, "fp8"],
                    help="fp8 = w8a8 e4m3fn projections (reported as dtype fp8; the headline is bf16)")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="fp8 = e4m3fn KV cache (reported in dtype; the headline is bf16)")
    ap.add_argument("--num-gpu-blocks", type=int, default=None)
    ap.add_argument("--gpu-mem-util", type=float, default=None,
                    help="device-memory fraction of aggregated / decode engines (default 0.9)")
    ap.add_argument("--prefill-gpu-mem-util", type=float, default=None,
                    help="N > 1: device-memory fraction of prefill engines (default 0.5; a TP1 70B prefill rank "
                         "needs ~0.9, as the reference's 4P(TP1) layout passes)")
    ap.add_argument("--prefill-max-seqs", type=int, default=32, help="N > 1: request slots of prefill engines")
    ap.add_argument("--p2p-backend", default="nccl", choices=["nccl", "gloo", "ipc"],
                    help="gloo = host-staged KV transfer (lets >1 rank share one GPU for functional tests); "
                         "ipc = one-sided WRITE (and prefix READ) through mappings of the decode caches (prefill "
                         "TP 1; works on one shared GPU too); never chosen implicitly")
    a = ap.parse_args(argv)
    if a.verify_tokens is None:
        a.verify_tokens = 2 if a.gpus > 1 and a.mode == "disagg" else 0
    if a.iters_per_step is None:
        a.iters_per_step = max(1, a.osl // 5)
    if a.max_batched_tokens is None:
        a.max_batched_tokens = SD["max_num_batched_tokens"] if a.policy == "chunked" else 16384
    return a


def log(msg):
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def run_aggregated(args, dev):
    import torch

    from dynamo_exp_amd.bench.serving import LoadGen, PromptGen, ServingWindow, drive
    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine

    cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=args.isl + args.osl + 64,
                       max_num_seqs=max(args.concurrency, 1), max_num_batched_tokens=args.max_batched_tokens,
                       max_prefill_streak=args.max_prefill_streak, use_cuda_graph=not args.no_graph,
                       chunked_prefill=args.policy == "chunked", device=str(dev), seed=args.seed,
                       quantization=args.quantization, min_prefill_tokens=args.min_prefill_tokens,
                       kv_cache_dtype=args.kv_cache_dtype,
                       max_prefill_delay=args.max_prefill_delay, num_gpu_blocks=args.num_gpu_blocks,
                       prefill_hold_min_decode=args.prefill_hold_min_decode,
                       prefill_hold_partial=args.prefill_hold_partial,
                       prefill_whole_prompts=bool(args.prefill_whole_prompts),
                       gpu_memory_utilization=args.gpu_mem_util or 0.90)
    if args.qps is not None:
        cfg.max_num_seqs = 256
    t0 = time.time()
    eng = LLMEngine(cfg)
    gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256) if s <= cfg.max_num_seqs]
    if cfg.max_num_seqs not in gs:
        gs.append(cfg.max_num_seqs)
    eng.runner.cfg.graph_sizes = tuple(gs)
    cap = eng.warmup()
    if args.gemm_report:
        with open(args.gemm_report, "w") as f:
            json.dump({"decode": eng.gemm_report, "prefill": eng.prefill_gemm_report}, f, indent=1)
    log(f"engine ready in {time.time() - t0:.1f}s (graphs {cap:.1f}s), kv blocks {eng.runner.num_blocks}")
    win = ServingWindow()
    load = LoadGen(lambda rid, p, sp, cb: eng.add_request(rid, p, sp, on_output=cb),
                   PromptGen(args.seed, args.isl, eng.model_cfg.vocab_size), args.osl, win, seed=args.seed)
    if args.qps is not None:
        load.start_open(args.qps)
    else:
        load.start_closed(args.concurrency)
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    mix = drive(eng, load, win, args, sync, log=log)
    if getattr(eng, "step_sizes", None):  # DX_STEP_SIZES=1 (incl. warm-up steps)
        import numpy as np

        t = np.array([n for n, _ in eng.step_sizes])
        log(f"prefill/mixed step tokens: n {len(t)} mean {t.mean():.0f} p10/25/50/75/90 "
            f"{np.percentile(t, [10, 25, 50, 75, 90]).round().tolist()} per-1024 bucket {np.bincount(t // 1024).tolist()}")
    log("engine timing (s, incl. warmup): " + str({k: round(v, 3) for k, v in eng.timing.items()}) +
        " runner: " + str({k: round(v, 3) if isinstance(v, float) else v for k, v in eng.runner.timing.items()}))
    extra = {"engine_iters": mix["steps"], "prefill_iters": mix["prefill_steps"],
             "decode_iters": mix["decode_steps"], "mixed_iters": mix["mixed_steps"],
             "prefill_step_tokens_mean": round(mix["prefill_step_tokens"] /
                                               max(1, mix["mixed_steps"] + mix["prefill_steps"]), 1)}
    qwin = None
    qps = qps_for_segment(args, win, 1.0)
    if qps:
        from dynamo_exp_amd.bench.serving import fixed_qps_segment

        load.stop()
        for rid in list(eng.requests):  # the closed loop is over: start the open loop from an idle engine
            eng.abort(rid)
        qwin = fixed_qps_segment(eng, lambda rid, p, sp, cb: eng.add_request(rid, p, sp, on_output=cb),
                                 PromptGen(args.seed + 77, args.isl, eng.model_cfg.vocab_size), args.osl, qps,
                                 args.qps_seconds, sync=sync, seed=args.seed + 7, log=log)
        extra["qps_segment"] = {"qps": round(qps, 3), "seconds": args.qps_seconds}
    return win, extra, qwin


def remote_frac_adder(eng, frac: float, seed: int):
    """--remote-frac q: (add, service) for LoadGen / drive.  A request is
    'remotely prefilled' with probability q: the scheduler allocates its
    blocks and parks it (on_remote_prefill), and service() -- before every
    engine iteration -- completes it as if its KV had landed from a prefill
    GPU, with a first token.  The KV bytes are not computed (decode cost does
    not depend on their values), the P->D unpack (~0.1 ms per ISL-3000
    request) is not charged."""
    import random

    rng = random.Random(seed)
    ready: list = []
    tok = min(1000, eng.model_cfg.vocab_size - 1)  # any token id: the first token a prefill GPU would send
    if frac > 0:
        eng.scheduler.on_remote_prefill = lambda r: ready.append(r.request_id)

    def add(rid, p, sp, cb):
        eng.add_request(rid, p, sp, on_output=cb, remote_prefill=frac > 0 and rng.random() < frac)

    def service():
        while ready:
            eng.finish_remote_prefill(ready.pop(), tok, 0.0)

    return add, service


def run_sweep(args, dev) -> dict:
    """--sweep: the reference's genai-perf concurrency sweep on one engine
    (perf.sh:17-54 sweeps 1..256 and compares throughput/GPU at matched
    tok/s/user; docs/architecture.md:57-61).  Per point: output tok/s of the
    GPU, tok/s per user (1000 / mean inter-token gap of the streams in the
    window), TTFT and ITL."""
    import torch

    from dynamo_exp_amd.bench.serving import LoadGen, PromptGen, ServingWindow, drive
    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine

    points = sorted({int(c) for c in args.sweep.split(",") if c.strip()})
    cmax = max(points)
    cfg = EngineConfig(model=args.model, block_size=args.block_size, max_model_len=args.isl + args.osl + 64,
                       max_num_seqs=cmax, max_num_batched_tokens=args.max_batched_tokens,
                       max_prefill_streak=args.max_prefill_streak, use_cuda_graph=not args.no_graph,
                       chunked_prefill=args.policy == "chunked", device=str(dev), seed=args.seed,
                       quantization=args.quantization, min_prefill_tokens=args.min_prefill_tokens,
                       kv_cache_dtype=args.kv_cache_dtype, max_prefill_delay=args.max_prefill_delay,
                       num_gpu_blocks=args.num_gpu_blocks, prefill_hold_min_decode=args.prefill_hold_min_decode,
                       prefill_hold_partial=args.prefill_hold_partial,
                       prefill_whole_prompts=bool(args.prefill_whole_prompts),
                       gpu_memory_utilization=args.gpu_mem_util or 0.90)
    eng = LLMEngine(cfg)
    gs = [s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256) if s <= cmax]
    if cmax not in gs:
        gs.append(cmax)
    eng.runner.cfg.graph_sizes = tuple(gs)
    eng.warmup()
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    out = []
    add, service = remote_frac_adder(eng, args.remote_frac, args.seed + 99)
    for i, c in enumerate(points):
        win = ServingWindow()
        load = LoadGen(add, PromptGen(args.seed + 17 * i, args.isl, eng.model_cfg.vocab_size), args.osl, win,
                       rid_prefix=f"c{c}-", seed=args.seed + i)
        load.start_closed(c)
        drive(eng, load, win, args, sync, service=service, log=log)
        load.stop()
        for rid in list(eng.requests):
            eng.abort(rid)
        while eng.has_unfinished():  # drain the aborted batch in flight
            service()
            eng.step()
        eng.kv.reset_prefix_cache()
        sm = win.summary()
        tps = win.gen / win.elapsed if win.elapsed > 0 else 0.0
        # tok/s/user from the mean gap between a stream's tokens over every
        # delivery in the window (prefill stalls included, like genai-perf's
        # per-request ITL), not only the few requests that complete in it
        itl = sm["itl_mean_ms"]
        pt = {"concurrency": c, "tok_s_gpu": round(tps, 1), "tok_s_user": round(1000.0 / itl, 2) if itl else None,
              **sm,
              "window_s": round(win.elapsed, 2)}
        log(f"sweep C={c}: {pt}")
        out.append(pt)
    role = "aggregated (agg-tp1)" if not args.remote_frac else f"decode role, remote-prefill fraction {args.remote_frac}"
    return {"metric": f"concurrency sweep, {MODEL_NAMES.get(args.model, args.model)} {role}",
            "n_gpus": 1, "remote_frac": args.remote_frac,
            "dtype": ("fp8-w8a8" if args.quantization == "fp8" else "bf16") + ("+fp8-kv" if args.kv_cache_dtype == "fp8" else ""),
            "data": "synthetic (random-token prompts, random-init weights of the real architecture)",
            "config": {"isl": args.isl, "osl": args.osl, "steps": args.steps, "warmup": args.warmup,
                       "iters_per_step": args.iters_per_step, "policy": args.policy,
                       "prefill_batching": [args.min_prefill_tokens, args.max_prefill_delay,
                                            args.prefill_hold_min_decode]},
            "points": out}


def qps_for_segment(args, win, share: float) -> float:
    """Requests/s of the fixed-QPS segment for one engine owning `share`
    GPUs' worth of load: --qps-segment per GPU, or 80 % of the rate the
    closed loop sustained; 0 = no segment (open-loop runs, or asked off)."""
    from dynamo_exp_amd.bench.serving import closed_loop_request_rate

    if args.qps is not None or args.qps_segment == 0:
        return 0.0
    if args.qps_segment:
        return args.qps_segment * share
    return 0.8 * closed_loop_request_rate(win, args.osl)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(args, argv) -> int:
    """`--gpus N` without a launcher: start N rank processes through
    torch.distributed.run (127.0.0.1 rendezvous) and return their status.
    This process never touches the GPU (no torch import here)."""
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    if args.p2p_backend == "gloo" and not args.cpu:
        # ranks sharing one GPU: fewer hardware queues per process, so the
        # ranks' queues all stay mapped instead of being time-sliced (the
        # supervisor caps worker processes the same way, sdk/serve.py)
        env["GPU_MAX_HW_QUEUES"] = str(min(2, int(env.get("GPU_MAX_HW_QUEUES") or 2)))
    return subprocess.call(cmd, env=env)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.sweep and args.gpus == 1:
        if world != 1:
            print("[bench] --sweep with --gpus 1 runs one process", file=sys.stderr)
            sys.exit(2)
        import torch

        dev = torch.device("cpu") if args.cpu else torch.device("cuda", 0)
        print(json.dumps(run_sweep(args, dev)), flush=True)
        return
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    # watchdog: a wedged multi-rank run dumps every thread's stack and exits
    # instead of holding the node (default 25 min for N > 1)
    dump_after = os.environ.get("DX_DUMP_AFTER") or ("1500" if world > 1 else None)
    if dump_after:
        import faulthandler

        faulthandler.dump_traceback_later(float(dump_after), exit=True)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    server = None
    if world > 1 and rank == 0 and args.mode == "disagg":  # control plane child process, before any GPU call
        from dynamo_exp_amd.disagg.bench_disagg import start_control_plane

        server = start_control_plane()
    import torch

    if args.cpu:
        dev = torch.device("cpu")
    else:
        local = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    extra: dict = {}
    if world > 1 and args.mode == "agg":
        from dynamo_exp_amd.bench.dp import run_data_parallel

        win, extra, qwin = run_data_parallel(args, dev, rank, world)
        parallelism = extra.pop("parallelism")
    elif world > 1:
        from dynamo_exp_amd.disagg.bench_disagg import run_disaggregated

        win, extra, qwin = run_disaggregated(args, dev, rank, world, server=server)
        parallelism = extra.pop("parallelism")
    else:
        win, extra, qwin = run_aggregated(args, dev)
        parallelism = "agg-tp1"
    if rank == 0 and extra.get("sweep_points") is not None:  # N > 1 --sweep: one JSON of the points
        print(json.dumps({"metric": f"concurrency sweep, {MODEL_NAMES.get(args.model, args.model)} {parallelism}",
                          "n_gpus": world, "dtype": "bf16", "data": "synthetic (random-token prompts, random-init "
                          "weights of the real architecture)",
                          "config": {"isl": args.isl, "osl": args.osl, "steps": args.steps, "warmup": args.warmup,
                                     "iters_per_step": args.iters_per_step, "parallelism": parallelism,
                                     **{k: v for k, v in extra.items() if k != "sweep_points"}},
                          "points": extra["sweep_points"]}), flush=True)
        return
    if rank == 0:
        elapsed = win.elapsed
        value = win.gen / elapsed if elapsed > 0 else 0.0
        at_qps = {}
        if qwin is not None:
            qs = qwin.summary()
            at_qps = {"qps": extra.get("qps_segment", {}).get("qps"),
                      "ttft_p50_ms_at_qps": qs["ttft_p50_ms"], "ttft_p99_ms_at_qps": qs["ttft_p99_ms"],
                      "itl_p50_ms_at_qps": qs["itl_p50_ms"], "requests_at_qps": len(qwin.ttft),
                      "output_tok_s_at_qps": round(qwin.gen / qwin.elapsed, 1) if qwin.elapsed > 0 else None}
        out = {
            "metric": metric_label(args.model, parallelism),
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(1, args.steps) * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp8-w8a8" if args.quantization == "fp8" else "bf16") +
                     ("+fp8-kv" if args.kv_cache_dtype == "fp8" else ""),
            "data": "synthetic (random-token prompts, random-init weights of the real architecture)",
            **win.summary(),
            **at_qps,
            "output_tokens": win.gen,
            "elapsed_s": round(elapsed, 3),
            "config": {
                "model": MODEL_NAMES.get(args.model, args.model),
                "global_batch": args.concurrency * world if args.qps is None else None,
                "seq_len": args.isl + args.osl,
                "isl": args.isl,
                "osl": args.osl,
                "load": (f"closed-loop C={args.concurrency}/GPU" if args.qps is None
                         else f"open-loop Poisson {args.qps} req/s/GPU"),
                "iters_per_step": args.iters_per_step,
                "policy": args.policy,
                "max_batched_tokens": args.max_batched_tokens,
                "prefill_batching": [args.min_prefill_tokens, args.max_prefill_delay, args.prefill_hold_min_decode],
                **({"prefill_hold_partial": args.prefill_hold_partial} if args.prefill_hold_partial else {}),
                **({"prefill_whole_prompts": 1} if args.prefill_whole_prompts else {}),
                "parallelism": parallelism,
                **extra,
            },
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
