"""Planner benchmark (reference docs/guides/planner_benchmark/benchmark_planner.md:
static 2P2D vs the local planner under a sinusoidal request rate, ISL 3000 /
OSL 150; the reference reports average sequence latency 18.5 -> 12.4 s and
2756 -> 2546 GPU-seconds on 8x H100).

Runs the real disaggregated serving graph -- `dynamo serve` supervisor,
OpenAI frontend, processor, decode workers, prefill workers, control-plane
prefill queue, planner with LocalConnector (scale-up = new watcher on a free
GPU, scale-down = lease revoke + drain) -- with `engine: sim` workers: the
MI355X timing model of Llama-3-8B TP1 (engine/sim.py, calibrated to
profiles/r2_role_capacities.txt), so it runs on CPU.  8 virtual GPUs
(DX_NUM_GPUS=8).  Load: tools/loadgen.py --trace sin (Poisson arrivals at
rate(t) = mid + amp sin(2 pi t / period)).

GPU-seconds = integral over the run of the GPUs held by prefill + decode
workers, sampled every second by the planner's metrics log (the static run
uses the planner in --no-operation mode as its observer, like the reference).

    python tools/planner_bench.py --mode static --prefill 2 --decode 2 --out profiles/x_static.json
    python tools/planner_bench.py --mode planner --prefill 1 --decode 1 --out profiles/x_planner.json
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

import httpx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gpu_seconds(log_path: str, t_from: float, t_to: float) -> tuple[float, list]:
    """Integrate (n_prefill + n_decode) over [t_from, t_to] (planner-log clock)."""
    pts = []
    with open(log_path) as f:
        for line in f:
            e = json.loads(line)
            if e.get("kind") == "metrics":
                pts.append((e["t"], e["n_prefill"] + e["n_decode"], e))
    total = 0.0
    for (t0, g, _), (t1, _, _) in zip(pts, pts[1:]):
        lo, hi = max(t0, t_from), min(t1, t_to)
        if hi > lo:
            total += g * (hi - lo)
    return total, pts


def start_graph(config: str, graph: str, prefill: int, decode: int, operate: bool, planner: dict,
                extra: list | None = None) -> tuple:
    """Launch `dynamo serve` with the local planner on 8 virtual GPUs and wait
    until a request round-trips.  Returns (proc, url, planner_log, offset),
    offset = wall-clock minus planner-log time."""
    work = tempfile.mkdtemp(prefix="dx_planner_bench_")
    cp_port, http_port = _free(), _free()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=work, DYN_LOG="warning", DX_NUM_GPUS="8")
    log_dir = os.path.join(work, "planner")
    cmd = [sys.executable, "-m", "dynamo_exp_amd.sdk.serve", graph, "-f", config,
           f"--Frontend.port={http_port}", f"--Worker.ServiceArgs.workers={decode}",
           f"--PrefillWorker.ServiceArgs.workers={prefill}",
           f"--Planner.no-operation={'false' if operate else 'true'}", f"--Planner.log-dir={log_dir}",
           "--enable-local-planner", "--control-plane", f"127.0.0.1:{cp_port}"]
    cmd += [f"--Planner.{k}={v}" for k, v in planner.items()]
    cmd += list(extra or [])
    proc = subprocess.Popen(cmd, cwd=os.path.join(ROOT, "examples", "llm"), env=env, start_new_session=True,
                            stdout=open(os.path.join(work, "serve.log"), "w"), stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{http_port}"
    try:
        t0 = time.time()
        while True:
            if proc.poll() is not None:
                raise RuntimeError(f"serve exited: see {work}/serve.log")
            try:
                r = httpx.post(f"{url}/v1/completions", timeout=30, json={
                    "model": "llama3-8b", "prompt": "warm up " * 300, "max_tokens": 4, "nvext": {"ignore_eos": True}})
                if r.status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            if time.time() - t0 > 300:
                raise RuntimeError("graph not ready after 300 s")
            time.sleep(1.0)
        plog = os.path.join(log_dir, "planner.jsonl")
        while not os.path.exists(plog) or os.path.getsize(plog) == 0:
            time.sleep(0.5)
        # planner "t" is relative to its own start; align by the last entry read
        with open(plog) as f:
            last_t = max(json.loads(l)["t"] for l in f)
        return proc, url, plog, time.time() - last_t
    except BaseException:
        stop_graph(proc)
        raise


def stop_graph(proc) -> None:
    try:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(60)
    except Exception:
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except Exception:
            pass


def planner_actions(plog: str, t0: float = 0.0) -> list[dict]:
    out = []
    with open(plog) as f:
        for line in f:
            e = json.loads(line)
            if e.get("kind") == "adjust" and e.get("actions"):
                out.append({"t": round(e["t"] - t0, 1), "actions": e["actions"]})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["static", "planner"], required=True)
    ap.add_argument("--prefill", type=int, default=2)
    ap.add_argument("--decode", type=int, default=2)
    ap.add_argument("--min-rate", type=float, default=5.0)
    ap.add_argument("--max-rate", type=float, default=20.0)
    ap.add_argument("--period", type=float, default=150.0)
    ap.add_argument("--duration", type=float, default=600.0)
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--adjustment-interval", type=float, default=10.0)
    ap.add_argument("--planner-args", default="", help="extra Planner k=v overrides, comma separated")
    ap.add_argument("--config", default="configs/disagg_planner_sim.yaml")
    ap.add_argument("--graph", default="graphs.disagg_router:Frontend")
    ap.add_argument("--client", choices=["httpx", "raw"], default="raw",
                    help="load generator client (raw: bare asyncio HTTP/1.1, keeps an open-loop schedule at 60 req/s)")
    ap.add_argument("--slowdown", type=float, default=1.0,
                    help="sim workers as a GPU k times slower than the MI355X model (the overload regime of the "
                         "reference's H100 run; VERDICT r3 next #6)")
    ap.add_argument("--gpu-gb", type=float, default=288.0, help="sim workers' device memory (KV pool), e.g. 80")
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)

    planner = {"adjustment-interval": a.adjustment_interval}
    planner.update(dict(kv.split("=", 1) for kv in a.planner_args.split(",") if kv))
    extra = [f"--{c}.sim-slowdown={a.slowdown}" for c in ("Worker", "PrefillWorker")]
    extra += [f"--{c}.sim-gpu-gb={a.gpu_gb}" for c in ("Worker", "PrefillWorker")]
    proc, url, plog, offset = start_graph(a.config, a.graph, a.prefill, a.decode, a.mode == "planner", planner, extra)
    try:
        print(f"[planner_bench] graph ready ({a.mode}, {a.prefill}P{a.decode}D), running the trace", flush=True)
        t_start = time.time()
        sys.path.insert(0, ROOT)
        from tools import loadgen

        res = loadgen.main(["--url", url, "--model", "llama3-8b", "--isl", str(a.isl), "--osl", str(a.osl),
                            "--trace", "sin", "--min-rate", str(a.min_rate), "--max-rate", str(a.max_rate),
                            "--period", str(a.period), "--duration", str(a.duration), "--isl-unit", "chars",
                            "--timeout", "900", "--client", a.client])[0]
        t_end = time.time()
        time.sleep(2.0)
        gs, pts = gpu_seconds(plog, t_start - offset, t_end - offset)
        trace = [{"t": round(p[0] - (t_start - offset), 1), "gpus": p[1], "prefill_queue": p[2]["prefill_queue"],
                  "kv_load": round(p[2]["kv_load"], 4), "n_prefill": p[2]["n_prefill"], "n_decode": p[2]["n_decode"]}
                 for p in pts if t_start - offset <= p[0] <= t_end - offset]
        adjust = planner_actions(plog, t_start - offset)
        out = {"mode": a.mode, "start": f"{a.prefill}P{a.decode}D", "engine": "sim (MI355X Llama-3-8B TP1 model)",
               "sim_slowdown": a.slowdown, "sim_gpu_gb": a.gpu_gb,
               "config": a.config, "graph": a.graph, "planner": planner,
               "trace": {"kind": "sin", "min_rate": a.min_rate, "max_rate": a.max_rate, "period": a.period,
                         "duration": a.duration, "isl": a.isl, "osl": a.osl},
               "avg_sequence_latency_s": round(res["latency_mean_ms"] / 1000, 3) if res.get("latency_mean_ms") else None,
               "gpu_seconds": round(gs, 1), "wall_s": round(t_end - t_start, 1), "loadgen": res,
               "planner_actions": adjust, "gpu_timeline_every_10s": trace[::10]}
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps({k: out[k] for k in ("mode", "start", "avg_sequence_latency_s", "gpu_seconds", "wall_s")}),
              flush=True)
    finally:
        stop_graph(proc)


if __name__ == "__main__":
    main()
