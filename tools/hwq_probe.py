#!/usr/bin/env python3
"""Which HIP streams share a hardware queue?  (P->D data-plane hazard probe.)

An RCCL receive is a kernel that holds its stream's hardware (AQL) queue until
the matching send runs.  HIP maps a process's streams onto GPU_MAX_HW_QUEUES
queues, so a kernel on another stream that landed on the same queue waits
behind the spin.  This probe measures the mapping
instead of guessing it: for a candidate compute stream C and each other
stream S, it parks a 300 ms `spin_for` kernel on S (the stand-in of a
spinning receive, csrc/kernels/wire_standin.hip) and times a tiny kernel on
C.  ~0.1 ms = separate queues; ~300 ms = C is stuck behind S.

Scenarios (each in a fresh process, so queue assignment starts clean):
  null    C = the legacy default stream, S = 8 normal-priority streams
  pool    C = a torch pool stream, S = 8 more torch pool streams
  high    C = a high-priority stream, S = 8 normal-priority streams
  high4   C = a high-priority stream, S = 3 more high-priority + 8 normal
  cumask  C = a full-CU-mask stream, S = 8 normal-priority streams

Decode-graph scenarios: a decode rank's exact stream set
-- the engine's high-priority compute / side / kv_copy / host_tier streams, a
high-priority TP-collective stream, and the RCCL point-to-point streams of a
4P4D decode rank (4 WRITE + 4 READ pair communicators + the world
communicator: 9 normal-priority pool streams, how ProcessGroupNCCL gets them)
-- with a spin_for kernel parked on every point-to-point stream, while the
captured decode graph replays on the compute stream:
  graph         the engine's compute stream (utils/streams.py)
  graph-legacy  round 5's compute stream, the legacy default stream

Usage: python tools/hwq_probe.py [--out gpurun_out/hwq_probe.json]
       python tools/hwq_probe.py --scenario graph
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCENARIOS = ("null", "pool", "high", "high4", "cumask")
GRAPH_SCENARIOS = ("graph", "graph-legacy")


def run_graph_scenario(name: str, spin_ms: int = 2500, replays: int = 20, batch: int = 64) -> dict:
    import torch

    from dynamo_exp_amd import _native
    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.utils import streams

    K = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = LLMEngine(EngineConfig(model="llama3-8b@8", device="cuda:0", block_size=64, max_model_len=2048,
                                 num_gpu_blocks=512, max_num_seqs=batch, graph_sizes=(batch,)))
    eng.warmup()  # captures the decode graph; this thread now runs on the compute stream
    g = eng.runner.graphs[batch]
    hp = [streams.stream(r, dev) for r in ("side", "kv_copy", "host_tier")]
    tp_rccl = torch.cuda.Stream(dev, priority=-1)  # ProcessGroupNCCL is_high_priority_stream (TP groups)
    p2p = [torch.cuda.Stream(dev) for _ in range(9)]  # ProcessGroupNCCL's default (normal) pool
    if name == "graph-legacy":
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
    comp = torch.cuda.current_stream(dev)
    x = torch.zeros(1024, device=dev)
    for s in hp + [tp_rccl] + p2p:
        with torch.cuda.stream(s):
            x.mul_(1.0)
    torch.cuda.synchronize()

    def replay_ms() -> tuple[float, float]:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(comp)
        for _ in range(replays):
            g.replay()
        b.record(comp)
        b.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / replays
        return max(a.elapsed_time(b) / replays, 0.0), wall

    for _ in range(3):
        replay_ms()
    idle = min(replay_ms()[1] for _ in range(5))
    for s in p2p:
        K.spin_for(spin_ms, 0, s.cuda_stream)
    time.sleep(0.05)
    t_launch = time.perf_counter()
    busy = [replay_ms()[1] for _ in range(5)]
    during = (time.perf_counter() - t_launch) * 1e3 < spin_ms  # the replays finished while the spins ran
    torch.cuda.synchronize()
    return {"scenario": name, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "stream_plan": streams.plan(dev), "n_p2p_spinning": len(p2p), "spin_ms": spin_ms,
            "replay_ms_idle": round(idle, 4), "replay_ms_spinning": round(min(busy), 4),
            "replay_ms_spinning_max": round(max(busy), 4), "ratio": round(max(busy) / idle, 4),
            "measured_while_spinning": during}


def run_scenario(name: str, spin_ms: int = 300) -> dict:
    import torch

    from dynamo_exp_amd import _native

    K = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lo, hi = K.stream_priority_range()
    x = torch.zeros(1024, device=dev)
    torch.cuda.synchronize()
    raw: list[int] = []

    def ext(h: int):
        raw.append(h)
        return torch.cuda.ExternalStream(h, device=dev)

    others: list[tuple[str, object]] = []
    if name == "null":
        comp = torch.cuda.default_stream(dev)
        others = [(f"normal{i}", ext(K.stream_create(0, 0))) for i in range(8)]
    elif name == "pool":
        comp = torch.cuda.Stream(dev)
        others = [(f"pool{i}", torch.cuda.Stream(dev)) for i in range(8)]
    elif name in ("high", "high4"):
        comp = ext(K.stream_create(hi, 0))
        if name == "high4":
            others = [(f"high{i}", ext(K.stream_create(hi, 0))) for i in range(3)]
        others += [(f"normal{i}", ext(K.stream_create(0, 0))) for i in range(8)]
    elif name == "cumask":
        comp = ext(K.stream_create(0, 1))
        others = [(f"normal{i}", ext(K.stream_create(0, 0))) for i in range(8)]
    else:
        raise SystemExit(f"unknown scenario {name}")

    def tiny_ms() -> float:
        ev = torch.cuda.Event()
        t0 = time.perf_counter()
        with torch.cuda.stream(comp):
            x.add_(1.0)
            ev.record()
        ev.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for _ in range(3):  # first launches on each stream pay setup
        tiny_ms()
        for _, s in others:
            with torch.cuda.stream(s):
                x.mul_(1.0)
        torch.cuda.synchronize()
    idle = min(tiny_ms() for _ in range(5))
    rows = []
    for label, s in others:
        K.spin_for(spin_ms, 0, s.cuda_stream)
        time.sleep(0.02)  # the spin is resident on its queue
        dt = tiny_ms()
        torch.cuda.synchronize()
        rows.append({"spinning": label, "compute_kernel_ms": round(dt, 3), "blocked": dt > spin_ms / 3})
    torch.cuda.synchronize()
    for h in raw:
        K.stream_destroy(h)
    return {"scenario": name, "priority_range": [lo, hi], "idle_ms": round(idle, 3),
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "rows": rows,
            "blocked_by": [r["spinning"] for r in rows if r["blocked"]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.scenario:
        fn = run_graph_scenario if a.scenario in GRAPH_SCENARIOS else run_scenario
        print(json.dumps(fn(a.scenario)), flush=True)
        return
    res = []
    for s in SCENARIOS + GRAPH_SCENARIOS:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--scenario", s], capture_output=True,
                           text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        out = json.loads(line[-1]) if line else {"scenario": s, "error": (r.stderr or "")[-2000:], "rc": r.returncode}
        print(json.dumps({k: v for k, v in out.items() if k != "rows"}), flush=True)
        res.append(out)
        if r.returncode != 0:
            break
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
