"""llmctl / http discovery / router / metrics / mock_worker (reference
launch/llmctl, components/{http,router,metrics}; the reference tests the
metrics + router path against `mock_worker`)."""
import argparse
import asyncio
import socket
import urllib.request

import pytest

from dynamo_exp_amd.cli import llmctl, metrics, mock_worker
from dynamo_exp_amd.cli.router import RouterService
from dynamo_exp_amd.kv import hashing
from dynamo_exp_amd.llm.discovery import ModelWatcher
from dynamo_exp_amd.llm.http_service import ModelManager
from dynamo_exp_amd.runtime import BackgroundServer, DistributedRuntime


@pytest.fixture(scope="module")
def cp():
    s = BackgroundServer().start()
    yield s.address
    s.stop()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_llmctl_and_model_watcher(cp):
    async def main():
        drt = await DistributedRuntime.create(cp, is_static=True)
        mm = ModelManager()
        w = await ModelWatcher(drt, mm).start()
        assert llmctl.main(["--control-plane", cp, "http", "add", "chat-models", "m1", "dynamo.Processor.chat"]) is None \
            or True
        await asyncio.sleep(0.2)
        assert "m1" in mm.chat and "m1" not in mm.completion
        await llmctl.add(drt.cp, "completion", "m1", "dynamo/Processor/completions", "random")
        await asyncio.sleep(0.2)
        assert "m1" in mm.completion
        rows = await llmctl.list_models(drt.cp, None)
        assert {(r["type"], r["endpoint"]) for r in rows} == {("chat", "dynamo/Processor/chat"),
                                                              ("completion", "dynamo/Processor/completions")}
        assert await llmctl.remove(drt.cp, "chat-models", "m1") == 1
        await asyncio.sleep(0.2)
        assert "m1" not in mm.chat and "m1" in mm.completion
        w._task.cancel()
        await drt.close(1)

    # llmctl.main runs its own event loop, so call it from a worker thread
    orig = llmctl.main

    def threaded(argv):
        import threading
        res = {}
        t = threading.Thread(target=lambda: res.setdefault("rc", orig(argv)))
        t.start()
        t.join()
        assert res["rc"] == 0

    llmctl.main = threaded
    try:
        asyncio.run(main())
    finally:
        llmctl.main = orig


def test_llmctl_rejects_bad_endpoint():
    with pytest.raises(ValueError):
        llmctl.parse_endpoint("ns.comp")


def _mw_args(cp, comp, seed):
    return argparse.Namespace(namespace="t", component=comp, endpoint="generate", interval=0.05, seed=seed,
                              control_plane=cp)


def test_mock_workers_metrics_exporter(cp):
    port = _free_port()

    async def main():
        readies = [asyncio.Event(), asyncio.Event()]
        tasks = [asyncio.create_task(mock_worker.serve(_mw_args(cp, "Mock", i), readies[i])) for i in range(2)]
        await asyncio.gather(*(r.wait() for r in readies))
        drt = await DistributedRuntime.create(cp, is_static=True)
        client = await drt.namespace("t").component("Mock").endpoint("generate").client()
        await client.wait_for_instances(timeout=10, n=2)
        out = [c async for c in await client.round_robin("hey")]
        assert "".join(out) == "hey"
        a = metrics.arg_parser().parse_args(["--namespace", "t", "--component", "Mock", "--port", str(port),
                                             "--host", "127.0.0.1", "--poll-interval", "0.1",
                                             "--control-plane", cp])
        stop = asyncio.Event()
        mt = asyncio.create_task(metrics.run(a, stop))
        await asyncio.sleep(0.3)
        await drt.namespace("t").publish("kv-hit-rate", {"worker_id": client.instance_ids()[0], "isl_blocks": 10,
                                                         "overlap_blocks": 4})
        await asyncio.sleep(0.5)
        body = await asyncio.to_thread(lambda: urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics").read())
        stop.set()
        pm = await mt
        text = body.decode()
        for name in ("llm_kv_blocks_active", "llm_kv_blocks_total", "llm_requests_active_slots",
                     "llm_requests_total_slots", "llm_load_avg", "llm_load_std", "llm_kv_hit_rate_percent"):
            assert name in text, name
        for wid in client.instance_ids():
            assert f'worker_id="{wid}"' in text
        assert 'llm_kv_hit_rate_percent{component="Mock",endpoint="load_metrics",worker_id="%d"} 40.0' % \
            client.instance_ids()[0] in text
        assert pm is not None
        for t in tasks:
            t.cancel()
        await drt.close(1)

    asyncio.run(main())


def test_router_service_prefers_prefix_owner(cp):
    async def main():
        readies = [asyncio.Event(), asyncio.Event()]
        tasks = [asyncio.create_task(mock_worker.serve(_mw_args(cp, "RW", 7 + i), readies[i])) for i in range(2)]
        await asyncio.gather(*(r.wait() for r in readies))
        drt = await DistributedRuntime.create(cp, is_static=True)
        svc = await RouterService(drt, "t", "RW", block_size=4).start()
        ids = await svc.client.wait_for_instances(timeout=10, n=2)
        owner = ids[1]
        toks = list(range(100, 132))
        seq = hashing.sequence_hashes(toks, 4)
        loc = hashing.block_hashes(toks, 4)
        comp = drt.namespace("t").component("RW")
        await comp.publish("kv_events", {"worker_id": owner, "event_id": 1, "stored_parent": None,
                                         "stored": [{"block_hash": s, "tokens_hash": h} for s, h in zip(seq, loc)],
                                         "removed": []})
        await asyncio.sleep(0.3)
        # equalize load so the overlap term decides
        for w in ids:
            svc.kv.metrics.update(w, {"kv_active_blocks": 0, "kv_total_blocks": 100, "request_active_slots": 0,
                                      "request_total_slots": 10})
        svc.kv.metrics.stale_after = 1e9
        out = [r async for r in svc.generate({"tokens": toks + [1, 2, 3]})]
        assert out[0]["worker_id"] == owner and out[0]["overlap_blocks"] == 8
        for t in tasks:
            t.cancel()
        await drt.close(1)

    asyncio.run(main())


def test_step_breakdown_tool(tmp_path):
    """tools/step_breakdown.py splits a kernel trace at each embedding launch
    and classifies steps with prefill attention as mixed."""
    import csv
    import sys

    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    from tools import step_breakdown

    rows = []
    t = 0
    for kind in ("decode", "mixed", "decode"):
        names = ["embedding_kernel", "Cijk_gemm", "decode_attn_kernel<4>", "rmsnorm_kernel"]
        if kind == "mixed":
            names += ["prefill_attn_v2_kernel<true>", "gemm256_kernel<1>"]
        for n in names:
            rows.append((n, t, t + 100_000))  # ns
            t += 110_000
    rows.append(("embedding_kernel", t, t + 10_000))  # closes the last step
    p = tmp_path / "trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)
    out = step_breakdown.breakdown(step_breakdown.load(str(p)))
    assert out["decode"]["steps"] == 2 and out["mixed"]["steps"] == 1
    assert out["mixed"]["families_ms"]["fused_mlp"] > 0 and "fused_mlp" not in out["decode"]["families_ms"]
    assert abs(out["decode"]["wall_ms"] - 0.44) < 1e-9 and out["decode"]["busy_ms"] < out["decode"]["wall_ms"]
    assert "GPU busy" in step_breakdown.report(out)
