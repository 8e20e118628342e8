#!/usr/bin/env python3
"""KV-aware routing vs random routing through the full serving graph.

Reproduces the reference's routing experiment (docs/architecture.md:78-87:
KV-aware routing 3x faster TTFT, 2x lower latency than random routing on
prefix-heavy traffic) with this framework's components: the OpenAI HTTP
frontend, the Processor (tokenise + route), the KV Router (radix indexer fed by
the workers' KV events + pushed load metrics) and N native-engine workers
(graphs.agg_router).  The workload is shared-prefix traffic
(tools/loadgen.py --prefix-groups): G groups of long shared prefixes +
unique suffixes, closed loop.  Each worker's KV pool holds only part of the
groups' prefixes, so the routing policy decides the prefix-cache hit rate.

The router mode is switched live through the control-plane key
`dynamo/processor/router` (as the reference's processor reads it from etcd);
each mode gets fresh prefix groups (different seed) so caches warmed by the
previous mode do not help it.

    python tools/router_bench.py --workers 2 --out gpurun_out/router_bench.json
(all workers share GPU 0 on a one-GPU box: DYN_DISABLE_AUTO_GPU_ALLOCATION=1)
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def wait_ready(url: str, model: str, deadline_s: float) -> None:
    import httpx

    t0 = time.time()
    last = t0
    while time.time() - t0 < deadline_s:
        if time.time() - last > 20:
            print(f"[router_bench] waiting for the graph ({time.time() - t0:.0f}s)", file=sys.stderr, flush=True)
            last = time.time()
        try:
            r = httpx.post(f"{url}/v1/chat/completions", timeout=60, json={
                "model": model, "messages": [{"role": "user", "content": "warm up"}], "max_tokens": 2,
                "nvext": {"ignore_eos": True}})
            if r.status_code == 200:
                return
        except httpx.HTTPError:
            pass
        time.sleep(1.0)
    raise TimeoutError("serving graph did not come up")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--num-gpu-blocks", type=int, default=640, help="per worker (limits the prefix cache)")
    ap.add_argument("--groups", type=int, default=16)
    ap.add_argument("--prefix-len", type=int, default=2048)
    ap.add_argument("--isl", type=int, default=2304)
    ap.add_argument("--osl", type=int, default=16)
    ap.add_argument("--concurrency", type=int, default=16)
    ap.add_argument("--requests-per-conc", type=int, default=10)
    ap.add_argument("--warmup-per-conc", type=int, default=2)
    ap.add_argument("--modes", default="random,kv", help="comma list of random, round-robin, kv, kv-load")
    ap.add_argument("--isl-unit", default="chars")
    ap.add_argument("--rate", type=float, default=None,
                    help="open loop: Poisson arrivals at this many requests/s for --duration s (instead of the "
                         "closed loop); each mode's first pass over the prefix groups is its own cache warm-up")
    ap.add_argument("--duration", type=float, default=120.0)
    ap.add_argument("--max-num-seqs", type=int, default=64, help="per worker")
    ap.add_argument("--cpu", action="store_true", help="CPU engines (plumbing test)")
    ap.add_argument("--ready-timeout", type=float, default=600)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    from tools import loadgen
    from dynamo_exp_amd.runtime.control_plane import SyncControlPlaneClient

    cp_port, http_port = free_port(), free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_LOG=os.environ.get("DYN_LOG", "warning"),
               DYN_DISABLE_AUTO_GPU_ALLOCATION="1", DYN_STATE_DIR=os.environ.get("DYN_STATE_DIR", "/tmp/dx_state"))
    args = [sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "graphs.agg_router:Frontend", "-f",
            "configs/agg_router.yaml", f"--Frontend.port={http_port}", f"--Frontend.served_model_name={a.model}",
            f"--Common.model={a.model}", f"--Common.block-size={a.block_size}",
            f"--Common.max-model-len={a.max_model_len}", f"--Worker.ServiceArgs.workers={a.workers}",
            f"--Worker.num-gpu-blocks={a.num_gpu_blocks}", f"--Worker.max-num-seqs={a.max_num_seqs}",
            "--Processor.router=random", "--control-plane", f"127.0.0.1:{cp_port}"]
    if a.cpu:
        args += ["--Worker.ServiceArgs.resources.gpu=0", "--Worker.device=cpu"]
    proc = subprocess.Popen(args, cwd=os.path.join(ROOT, "examples", "llm"), env=env, start_new_session=True)
    url = f"http://127.0.0.1:{http_port}"
    results = {}
    try:
        wait_ready(url, a.model, a.ready_timeout)
        cp = SyncControlPlaneClient(f"127.0.0.1:{cp_port}")
        # every worker registered (= warmed up) before timing: a worker still
        # initialising shares the GPU with the measured ones
        t0 = time.time()
        while True:
            n = sum(1 for k, _ in cp.get_prefix("dynamo/components/Worker/") if "/generate:" in k)
            if n >= a.workers or time.time() - t0 > a.ready_timeout:
                break
            time.sleep(1.0)
        print(f"[router_bench] {n} workers registered", file=sys.stderr, flush=True)
        for i, mode in enumerate(a.modes.split(",")):
            cp.put("dynamo/processor/router", mode.encode())
            time.sleep(0.5)
            load = (["--trace", "sin", "--min-rate", str(a.rate), "--max-rate", str(a.rate), "--duration",
                     str(a.duration), "--client", "raw", "--timeout", "900"] if a.rate else
                    ["--concurrency", str(a.concurrency), "--requests-per-conc", str(a.requests_per_conc),
                     "--warmup-per-conc", str(a.warmup_per_conc)])
            la = loadgen.main(["--url", url, "--model", a.model, "--isl", str(a.isl), "--osl", str(a.osl),
                               "--isl-unit", a.isl_unit, "--prefix-groups", str(a.groups),
                               "--prefix-len", str(a.prefix_len), "--seed", str(1000 + i)] + load)
            results[mode] = la[0]
            print(f"[router_bench] {mode}: {json.dumps(la[0])}", file=sys.stderr, flush=True)
        cp.close()
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
    keys = ("model", "workers", "num_gpu_blocks", "groups", "prefix_len", "isl", "osl", "concurrency",
            "requests_per_conc", "rate", "duration", "max_num_seqs")
    out = {"workload": {k: getattr(a, k) for k in keys},
           "modes": results}
    if "random" in results and "kv" in results:
        r, k = results["random"], results["kv"]
        out["kv_vs_random"] = {
            "ttft_mean_speedup": round(r["ttft_mean_ms"] / k["ttft_mean_ms"], 2) if k.get("ttft_mean_ms") else None,
            "ttft_p50_speedup": round(r["ttft_p50_ms"] / k["ttft_p50_ms"], 2) if k.get("ttft_p50_ms") else None,
            "latency_p50_speedup": round(r["latency_p50_ms"] / k["latency_p50_ms"], 2) if k.get("latency_p50_ms") else None,
            "throughput_ratio": round(k["output_tok_s"] / r["output_tok_s"], 2) if r.get("output_tok_s") else None}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
