"""Load generator against a live frontend (echo engine, CPU)."""
import os
import socket
import subprocess
import sys
import time

import httpx
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_loadgen_sweep_and_sin_trace():
    import loadgen

    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_TOKEN_ECHO_DELAY_MS="1", DYN_LOG="warning")
    proc = subprocess.Popen([sys.executable, "-m", "dynamo_exp_amd.cli.run", "in=http", "out=echo_core",
                             "--model-path", "tiny", "--model-name", "tiny", "--http-port", str(port)], env=env,
                            start_new_session=True)
    try:
        for _ in range(200):
            try:
                if httpx.get(f"http://127.0.0.1:{port}/v1/models", timeout=2).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.2)
        url = f"http://127.0.0.1:{port}"
        pts = loadgen.main(["--url", url, "--model", "tiny", "--isl", "20", "--osl", "8", "--concurrency", "1,4",
                            "--requests-per-conc", "3", "--warmup-per-conc", "1"])
        assert [p["concurrency"] for p in pts] == [1, 4]
        for p in pts:
            assert p["ok"] == p["requests"] and p["output_tok_s"] > 0 and p["ttft_p50_ms"] is not None
        sin = loadgen.main(["--url", url, "--model", "tiny", "--isl", "10", "--osl", "4", "--trace", "sin",
                            "--min-rate", "5", "--max-rate", "20", "--period", "2", "--duration", "2"])[0]
        assert sin["ok"] > 5 and sin["ok"] == sin["requests"]
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)


def test_sim_engine_batched_delivery():
    """SimLLMEngine through AsyncLLMEngine (per-step batched delivery): every
    stream gets exactly max_tokens tokens and an abandoned stream is aborted."""
    import asyncio

    from dynamo_exp_amd.engine.engine import AsyncLLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams
    from dynamo_exp_amd.engine.sim import SimLLMEngine

    sim = SimLLMEngine(decode_ms=1.0, prefill_tok_per_ms=1000.0)
    sim.host_ms = 0.0
    ae = AsyncLLMEngine(sim).start()

    async def one(n):
        toks, fin = [], None
        async for o in ae.generate(None, list(range(50)), SamplingParams(max_tokens=n, ignore_eos=True)):
            toks += o["token_ids"]
            fin = o["finish_reason"]
        return toks, fin

    async def cancelled():
        agen = ae.generate("c1", list(range(50)), SamplingParams(max_tokens=10_000, ignore_eos=True))
        got = 0
        async for o in agen:
            got += len(o["token_ids"])
            if got >= 3:
                break
        await agen.aclose()
        return got

    async def main():
        res = await asyncio.gather(*(one(5 + i) for i in range(16)), cancelled())
        return res

    try:
        res = asyncio.run(main())
        for i, (toks, fin) in enumerate(res[:16]):
            assert len(toks) == 5 + i and fin == "length"
        assert res[16] >= 3
        deadline = time.time() + 5
        while sim.has_pending_work() and time.time() < deadline:  # the abort reaches the engine thread
            time.sleep(0.01)
        assert not sim.has_pending_work()
    finally:
        ae.shutdown()


def test_prefix_groups_prompts():
    import random

    import loadgen

    loadgen.ISL_UNIT["unit"] = "chars"
    src = loadgen.PromptSource(random.Random(0), 120, groups=3, prefix_len=100)
    ps = [src() for _ in range(30)]
    assert all(len(p) == 120 for p in ps)
    assert len({p[:100] for p in ps}) == 3 and len(set(ps)) == 30
    loadgen.ISL_UNIT["unit"] = "words"


@pytest.mark.slow
def test_router_bench_cpu_plumbing():
    """tools/router_bench.py end to end on CPU engines: agg_router graph with 2
    workers, router mode switched live (random -> kv) over the control plane."""
    import json

    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "router_bench.py"), "--cpu", "--model", "tiny",
                          "--block-size", "16", "--max-model-len", "512", "--num-gpu-blocks", "120", "--groups", "4",
                          "--prefix-len", "160", "--isl", "200", "--osl", "3", "--concurrency", "3",
                          "--requests-per-conc", "2", "--warmup-per-conc", "1", "--ready-timeout", "240",
                          "--modes", "random,kv,kv-load"],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["modes"]["random"]["ok"] == 6 and res["modes"]["kv"]["ok"] == 6
    assert res["modes"]["kv-load"]["ok"] == 6  # least-KV-usage routing (kv_router.py:226-245)
    assert res["kv_vs_random"]["ttft_mean_speedup"] is not None
