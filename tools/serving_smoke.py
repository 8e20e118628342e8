"""GPU smoke of the full serving stack: `run in=http out=native` (single
process) and the `serve` agg graph (Frontend -> Processor -> Worker
processes), each driven with OpenAI HTTP requests; prints a JSON summary with
TTFT / latency of a few concurrent streaming requests."""
from __future__ import annotations

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


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def drive(port: int, model: str, n: int = 8, isl_words: int = 400, osl: int = 64) -> dict:
    async with httpx.AsyncClient(timeout=600) as c:
        for _ in range(600):
            try:
                r = await c.get(f"http://127.0.0.1:{port}/v1/models")
                if r.status_code == 200 and r.json()["data"]:
                    break
            except httpx.HTTPError:
                pass
            await asyncio.sleep(1)

        async def one(i):
            t0 = time.perf_counter()
            ttft = None
            n_chunks = 0
            async with c.stream("POST", f"http://127.0.0.1:{port}/v1/chat/completions", json={
                "model": model, "stream": True, "max_tokens": osl, "nvext": {"ignore_eos": True},
                "messages": [{"role": "user", "content": " ".join(f"word{i}_{k}" for k in range(isl_words))}]}) as r:
                async for line in r.aiter_lines():
                    if line.startswith("data: {"):
                        if ttft is None:
                            ttft = time.perf_counter() - t0
                        n_chunks += 1
            return {"ttft_ms": round(ttft * 1000, 1), "latency_ms": round((time.perf_counter() - t0) * 1000, 1),
                    "chunks": n_chunks}

        res = await asyncio.gather(*[one(i) for i in range(n)])
        r = await c.post(f"http://127.0.0.1:{port}/v1/completions",
                         json={"model": model, "prompt": "hello", "max_tokens": 8})
        unary = r.status_code
        m = (await c.get(f"http://127.0.0.1:{port}/metrics")).text if "metrics" else ""
    return {"requests": res, "unary_status": unary, "metrics_lines": len(m.splitlines())}


def run_single(model: str) -> dict:
    port = free_port()
    p = subprocess.Popen([sys.executable, "-m", "dynamo_exp_amd.cli.run", "in=http", "out=native", "--model-path",
                          model, "--http-port", str(port), "--max-model-len", "4096"], cwd=ROOT,
                         start_new_session=True)
    try:
        return asyncio.run(drive(port, "Llama-3-8B" if model == "llama3-8b" else model))
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(60)


def run_graph(model: str) -> dict:
    port, cp = free_port(), free_port()
    p = subprocess.Popen([sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "graphs.agg:Frontend", "-f",
                          "configs/agg.yaml", f"--Frontend.port={port}", f"--Frontend.served_model_name={model}",
                          f"--Common.model={model}", "--Common.max-model-len=4096", "--control-plane",
                          f"127.0.0.1:{cp}"], cwd=os.path.join(ROOT, "examples", "llm"),
                         env=dict(os.environ, PYTHONPATH=ROOT), start_new_session=True)
    try:
        return asyncio.run(drive(port, model))
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(60)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)


if __name__ == "__main__":
    model = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b"
    out = {"single_process": run_single(model), "serve_agg_graph": run_graph(model)}
    print(json.dumps(out, indent=1))
