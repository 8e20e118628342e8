"""The SERVED disaggregated graph on one MI355X with HIP engines (VERDICT r4
next #2): `dynamo serve graphs.disagg_router:Frontend` -- HTTP frontend ->
processor -> KV router -> decode worker -> prefill queue -> prefill worker ->
KV transfer -> decode -> SSE -- with Llama-3-8B at 8 layers, both workers on
the one GPU (half a GPU each), KV moved with the explicit `--kv-transport
host` (pinned-host staging over per-pair gloo groups; RCCL needs distinct
devices).  Reference: examples/llm/components/worker.py:180-229,
prefill_worker.py:118-159.

Checked: OpenAI streaming completions end with [DONE]; the prompts went
remote (the decode worker's KV-transfer histogram); the KV events reached the
router (a repeated prompt is routed with a prefix overlap, published on
kv-hit-rate); the prefill queue drained; greedy tokens equal those of
`graphs.agg:Frontend` (same preset weights, same kernels: the GEMM tuners are
off so both graphs pick the same kernels)."""
from __future__ import annotations

import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPTS = [f"request {i}: " + " ".join(f"w{(i * 37 + k) % 101}" for k in range(160)) for i in range(3)]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _serve(graph: str, cfg: str, extra: list[str], tag: str, tmp_path, model: str):
    cp_port, http_port = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=str(tmp_path / tag), DYN_LOG="info",
               DX_SKINNY="0", DX_PREFILL_TUNE="0", PYTHONUNBUFFERED="1")
    os.makedirs(tmp_path / tag, exist_ok=True)
    args = [sys.executable, "-m", "dynamo_exp_amd.sdk.serve", graph, "-f", cfg, f"--Frontend.port={http_port}",
            f"--Frontend.served_model_name={model}", f"--Common.model={model}", "--Common.block-size=64",
            "--Common.max-model-len=4096", "--control-plane", f"127.0.0.1:{cp_port}"] + extra
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log = open(os.path.join(ROOT, "gpurun_out", f"serve_{tag}.log"), "w")
    proc = subprocess.Popen(args, cwd=os.path.join(ROOT, "examples", "llm"), env=env, start_new_session=True,
                            stdout=log, stderr=subprocess.STDOUT)
    return proc, http_port, f"127.0.0.1:{cp_port}", log


def _stop(proc, log) -> None:
    try:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(60)
    except (subprocess.TimeoutExpired, ProcessLookupError):
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
    log.close()


def _stream(port: int, prompt: str, deadline: float, model: str) -> str:
    """One streaming greedy completion; returns the generated text.  Retries
    connection errors until the graph is up (or the deadline)."""
    import httpx

    body = {"model": model, "prompt": prompt, "max_tokens": 16, "temperature": 0, "stream": True,
            "nvext": {"ignore_eos": True}}
    last = None
    while time.time() < deadline:
        try:
            with httpx.stream("POST", f"http://127.0.0.1:{port}/v1/completions", json=body, timeout=120) as r:
                if r.status_code != 200:
                    last = f"HTTP {r.status_code}"
                    time.sleep(1.0)
                    continue
                lines = [ln for ln in r.iter_lines() if ln.startswith("data:")]
            if lines and "no instances for" in lines[-1]:  # the frontend is up before a downstream component
                last = lines[-1]
                time.sleep(1.0)
                continue
            assert lines and lines[-1].strip() == "data: [DONE]", lines[-3:]
            text = ""
            for ln in lines[:-1]:
                ch = json.loads(ln[5:])
                text += ch["choices"][0].get("text") or ""
            return text
        except (httpx.HTTPError, OSError) as e:
            last = repr(e)
            time.sleep(1.0)
    raise AssertionError(f"graph did not serve: {last}")


def _metric(port: int, name: str) -> float:
    import httpx

    tot = 0.0
    for ln in httpx.get(f"http://127.0.0.1:{port}/metrics", timeout=10).text.splitlines():
        if ln.startswith("#"):
            continue
        if name in ln.split("{")[0].split(" ")[0]:
            tot += float(ln.rsplit(" ", 1)[1])
    return tot


def _agg_then_disagg(tmp_path, model: str, gpu: str, transport: str):
    # ---- aggregated graph: the reference tokens
    proc, port, _, log = _serve("graphs.agg:Frontend", "configs/agg.yaml",
                                ["--Worker.num-gpu-blocks=1024", "--Worker.max-num-seqs=16",
                                 f"--Worker.ServiceArgs.resources.gpu={1 if gpu != '0' else 0}"], "agg", tmp_path, model)
    try:
        deadline = time.time() + 240
        want = [_stream(port, p, deadline, model) for p in PROMPTS + PROMPTS[:1]]
    finally:
        _stop(proc, log)
    assert all(want), want

    # ---- disaggregated graph with the KV router, both workers on the one GPU
    metrics_port = _free_port()
    extra = ["--Worker.ServiceArgs.workers=1", f"--Worker.ServiceArgs.resources.gpu={gpu}",
             "--PrefillWorker.ServiceArgs.workers=1", f"--PrefillWorker.ServiceArgs.resources.gpu={gpu}",
             "--Worker.num-gpu-blocks=1024", "--Worker.max-num-seqs=16", "--PrefillWorker.num-gpu-blocks=512",
             f"--Worker.kv-transport={transport}", f"--PrefillWorker.kv-transport={transport}",
             "--Worker.max-local-prefill-length=64", "--Worker.max-prefill-queue-size=8",
             f"--Worker.metrics-port={metrics_port}"]
    proc, port, cp, log = _serve("graphs.disagg_router:Frontend", "configs/disagg_router.yaml", extra, "disagg",
                                 tmp_path, model)
    try:
        from dynamo_exp_amd.disagg.prefill_queue import PrefillQueue
        from dynamo_exp_amd.llm.kv_router import KV_HIT_RATE_SUBJECT
        from dynamo_exp_amd.runtime.distributed import DistributedRuntime

        hits: list[dict] = []

        async def watch_and_run():
            deadline = time.time() + 420
            drt = None
            while drt is None:
                try:
                    drt = await DistributedRuntime.create(cp, is_static=True)
                except Exception:  # noqa: BLE001 -- the control plane is still starting
                    if time.time() > deadline:
                        raise
                    await asyncio.sleep(0.5)
            sub = await drt.namespace("dynamo").subscribe(KV_HIT_RATE_SUBJECT)

            async def pump():
                async for ev in sub:
                    hits.append(ev)

            t = asyncio.create_task(pump())
            got = []
            for p in PROMPTS + PROMPTS[:1]:  # one at a time: the same batch shapes as the aggregated run
                got.append(await asyncio.to_thread(_stream, port, p, deadline, model))
            await asyncio.sleep(0.5)
            qsize = await PrefillQueue(drt.cp, "prefill_queue").size()
            t.cancel()
            await drt.close(1)
            return got, qsize

        got, qsize = asyncio.run(watch_and_run())
        transfers = _metric(metrics_port, "kv_transfer_seconds_count")
        xfer_bytes = _metric(metrics_port, "kv_transfer_bytes")
    finally:
        _stop(proc, log)
    # the three distinct prompts were prefilled remotely and their KV moved
    assert transfers >= 3, transfers
    assert xfer_bytes > 0, xfer_bytes
    assert qsize == 0
    # KV events of the decode worker reached the router: the repeated prompt
    # was routed with a prefix overlap
    assert len(hits) >= 4, hits
    assert hits[-1]["overlap_blocks"] > 0, hits
    assert got == want, (got, want)


@pytest.mark.gpu
def test_served_disagg_router_graph_one_gpu(tmp_path):
    _agg_then_disagg(tmp_path, "llama3-8b@8", "0.5", "host")


@pytest.mark.gpu
def test_served_disagg_router_graph_one_gpu_one_sided(tmp_path):
    """The same served graph with `--kv-transport ipc`: the prefill worker
    writes straight into the decode worker's shared KV cache (disagg/
    kv_share.py), two processes on the one GPU."""
    _agg_then_disagg(tmp_path, "llama3-8b@8", "0.5", "ipc")


@pytest.mark.slow
def test_served_disagg_router_graph_cpu(tmp_path):
    """The same graph and checks with CPU engines (tiny preset, gloo links)."""
    _agg_then_disagg(tmp_path, "tiny", "0", "host")
