"""The planner against the real disaggregated serving graph (supervisor,
frontend, processor, KV-load router, control-plane prefill queue) with
simulated MI355X workers: a burst of long prompts backs up the prefill queue,
the planner adds a prefill worker (new watcher on a free virtual GPU), and
once the queue is empty it removes one again -- lease revoke, the prefill
worker stops pulling and drains (llm/workers.py PrefillWorker.run) -- with
no request lost (reference components/planner/test/load_test.sh: 1P1D ->
1P2D -> 1P1D, and local_connector.py:197-325)."""
import asyncio
import json
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.slow
def test_planner_scales_prefill_up_and_drains_down():
    import httpx

    from tools.planner_bench import planner_actions, start_graph, stop_graph

    planner = {"adjustment-interval": 3, "prefill-queue-scale-up-threshold": 2,
               "prefill-queue-scale-down-threshold": 0.2, "decode-kv-scale-up-threshold": 0.99,
               "decode-kv-scale-down-threshold": 0.0}
    proc, url, plog, _ = start_graph("configs/disagg_planner_sim.yaml", "graphs.disagg_router:Frontend", 1, 1,
                                     True, planner)
    try:
        async def burst(n):
            async with httpx.AsyncClient(timeout=300, limits=httpx.Limits(max_connections=n + 8)) as c:
                async def one(i):
                    r = await c.post(f"{url}/v1/completions", json={
                        "model": "llama3-8b", "prompt": f"{i} " + "x" * 6000, "max_tokens": 4,
                        "nvext": {"ignore_eos": True}})
                    return r.status_code
                return await asyncio.gather(*(one(i) for i in range(n)))

        codes = asyncio.run(burst(240))  # ~1.4M prompt tokens: ~15 s of one simulated prefill GPU
        t_burst_end = time.time()
        assert codes == [200] * 240
        adds = removes = 0
        while time.time() - t_burst_end < 90:
            acts = [a for e in planner_actions(plog) for a in e["actions"]]
            adds = sum(1 for a, c in acts if a == "add" and c == "PrefillWorker")
            removes = sum(1 for a, c in acts if a == "remove" and c == "PrefillWorker")
            if adds and removes:
                break
            time.sleep(2)
        assert adds >= 1, planner_actions(plog)
        assert removes >= 1, planner_actions(plog)
        # the graph still serves after the scale-down drain
        r = httpx.post(f"{url}/v1/completions", timeout=60, json={
            "model": "llama3-8b", "prompt": "y" * 3000, "max_tokens": 4, "nvext": {"ignore_eos": True}})
        assert r.status_code == 200, r.text
        with open(plog) as f:
            peak = max(e["n_prefill"] for e in map(json.loads, f) if e.get("kind") == "metrics")
        assert peak >= 2
    finally:
        stop_graph(proc)
