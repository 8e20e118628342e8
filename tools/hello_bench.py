#!/usr/bin/env python3
"""hello_world agg graph throughput (BASELINE config 1: plumbing, no GPU):
Frontend (FastAPI /generate) -> Middle -> Backend x2 over the in-tree control
plane + request plane; closed loop at several concurrencies, streamed
responses read to the end.  Reports requests/s and latency p50/p99."""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import time

import httpx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


async def run_point(url: str, conc: int, n: int) -> dict:
    import aiohttp  # lighter per request than httpx: keeps the client off the critical path

    lat = []
    conn = aiohttp.TCPConnector(limit=conc + 4)
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=30)) as c:
        async def worker(k):
            for i in range(n):
                t0 = time.perf_counter()
                async with c.post(f"{url}/generate", json={"text": f"hi {k} {i}"}) as r:
                    async for _ in r.content.iter_any():
                        pass
                    assert r.status == 200
                lat.append(time.perf_counter() - t0)
        for _ in range(2):  # warm connections / paths
            await worker(-1)
        lat.clear()
        t0 = time.perf_counter()
        await asyncio.gather(*(worker(k) for k in range(conc)))
        wall = time.perf_counter() - t0
    lat.sort()
    return {"concurrency": conc, "requests": len(lat), "req_s": round(len(lat) / wall, 1),
            "p50_ms": round(lat[len(lat) // 2] * 1e3, 2), "p99_ms": round(lat[int(len(lat) * 0.99)] * 1e3, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", default="1,8,32,64")
    ap.add_argument("--requests-per-conc", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cp_port, port = free_port(), free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_LOG="warning", DYN_STATE_DIR="/tmp/dx_hello_state")
    proc = subprocess.Popen([sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "hello_world:Frontend", "-f",
                             "config.yaml", f"--Frontend.port={port}", "--control-plane", f"127.0.0.1:{cp_port}"],
                            cwd=os.path.join(ROOT, "examples", "hello_world"), env=env, start_new_session=True)
    url = f"http://127.0.0.1:{port}"
    try:
        t0 = time.time()
        while time.time() - t0 < 120:
            try:
                if httpx.post(f"{url}/generate", json={"text": "x"}, timeout=5).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.5)
        time.sleep(2.0)  # both Backend workers registered
        pts = [asyncio.run(run_point(url, int(c), a.requests_per_conc)) for c in a.concurrency.split(",")]
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
    out = {"graph": "hello_world:Frontend (Frontend -> Middle -> Backend x2)", "points": pts}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
