"""SDK: config merging (mirrors deploy/dynamo/sdk/src/dynamo/sdk/tests/test_config.py),
graph links, dry-run, and an end-to-end `serve` of the 3-stage hello_world
graph (control plane + supervisor + 4 worker processes + FastAPI /generate)."""
import json
import os
import socket
import subprocess
import sys
import time

import httpx
import pytest

from dynamo_exp_amd.sdk.config import ServiceConfig, resolve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_as_args_with_common():
    cfg = ServiceConfig({
        "Common": {"model": "m", "block-size": 64, "shared": True},
        "Worker": {"common-configs": ["model", "block-size"], "block-size": 128, "remote-prefill": True,
                   "ServiceArgs": {"workers": 2}, "extra": {"a": 1}},
    })
    args = cfg.as_args("Worker")
    assert args[:2] == ["--model", "m"]
    assert "--block-size" in args and args[args.index("--block-size") + 1] == "128"
    assert "--remote-prefill" in args
    assert "--workers" not in args and "--shared" not in args
    assert json.loads(args[args.index("--extra") + 1]) == {"a": 1}
    assert cfg.as_args("Nope") == []


def test_resolve_overrides(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("A:\n  x: 1\n  ServiceArgs:\n    workers: 1\n")
    cfg = resolve(str(p), ["--A.x=5", "--A.ServiceArgs.workers=3", "--B.name=hi"])
    assert cfg == {"A": {"x": 5, "ServiceArgs": {"workers": 3}}, "B": {"name": "hi"}}


def test_graph_and_links():
    sys.path.insert(0, os.path.join(ROOT, "examples", "hello_world"))
    import hello_world as hw

    assert [s.name for s in hw.Frontend.graph()] == ["Frontend", "Middle", "Backend"]
    assert hw.Backend.workers == 2
    assert hw.Frontend.endpoints["generate"].is_api


def test_dry_run():
    out = subprocess.run([sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "hello_world:Frontend", "-f",
                          "config.yaml", "--dry-run", "--Backend.ServiceArgs.workers=3"],
                         cwd=os.path.join(ROOT, "examples", "hello_world"), capture_output=True, text=True,
                         timeout=120, env=dict(os.environ, PYTHONPATH=ROOT))
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert {s["name"]: s["workers"] for s in d["services"]} == {"Frontend": 1, "Middle": 1, "Backend": 3}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_e2e_hello_world(tmp_path):
    cp_port, http_port = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=str(tmp_path), DYN_LOG="warning")
    proc = subprocess.Popen([sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "hello_world:Frontend", "-f",
                             "config.yaml", f"--Frontend.port={http_port}", "--control-plane",
                             f"127.0.0.1:{cp_port}"], cwd=os.path.join(ROOT, "examples", "hello_world"), env=env,
                            start_new_session=True)
    try:
        body = None
        for _ in range(240):
            try:
                r = httpx.post(f"http://127.0.0.1:{http_port}/generate", json={"text": "hi"}, timeout=5)
                if r.status_code == 200:
                    body = r.text
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.5)
        assert body is not None, "graph did not come up"
        lines = [l for l in body.splitlines() if l]
        assert lines[0] == "Frontend: Middle: Backend: hi-earth-moon-mars"
        st = json.load(open(tmp_path / "inference.json"))
        assert set(st["watchers"]) == {"inference_Frontend", "inference_Middle", "inference_Backend"}
        assert len(st["watchers"]["inference_Backend"]["pids"]) == 2
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)


def _serve_llm_graph(tmp_path, graph, cfg, extra):
    cp_port, http_port = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=str(tmp_path), DYN_LOG="warning",
               DYN_TOKEN_ECHO_DELAY_MS="0")
    args = [sys.executable, "-m", "dynamo_exp_amd.sdk.serve", graph, "-f", cfg, f"--Frontend.port={http_port}",
            "--Frontend.served_model_name=tiny", "--Common.model=tiny", "--Common.block-size=16",
            "--Common.max-model-len=1024", "--Worker.num-gpu-blocks=300", "--Worker.ServiceArgs.resources.gpu=0",
            "--control-plane", f"127.0.0.1:{cp_port}"] + extra
    proc = subprocess.Popen(args, cwd=os.path.join(ROOT, "examples", "llm"), env=env, start_new_session=True)
    return proc, http_port


@pytest.mark.slow
@pytest.mark.parametrize("graph,cfg,extra", [
    ("graphs.agg:Frontend", "configs/agg.yaml", []),
    ("graphs.disagg:Frontend", "configs/disagg.yaml",
     ["--PrefillWorker.num-gpu-blocks=300", "--PrefillWorker.ServiceArgs.resources.gpu=0",
      "--Worker.max-local-prefill-length=5"]),
])
def test_e2e_llm_graph_cpu(tmp_path, graph, cfg, extra):
    proc, port = _serve_llm_graph(tmp_path, graph, cfg, extra)
    try:
        ok = None
        for _ in range(300):
            try:
                r = httpx.post(f"http://127.0.0.1:{port}/v1/chat/completions", timeout=30, json={
                    "model": "tiny", "messages": [{"role": "user", "content": "hello there"}], "max_tokens": 6,
                    "nvext": {"ignore_eos": True}})
                if r.status_code == 200:
                    ok = r.json()
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.5)
        assert ok is not None, "graph did not serve"
        assert ok["choices"][0]["finish_reason"] == "length"
        r = httpx.post(f"http://127.0.0.1:{port}/v1/chat/completions", timeout=30, json={
            "model": "tiny", "messages": [{"role": "user", "content": "stream please"}], "max_tokens": 5,
            "stream": True, "nvext": {"ignore_eos": True}})
        assert r.text.strip().endswith("data: [DONE]")
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)


@pytest.mark.slow
def test_e2e_disagg_skeleton(tmp_path):
    """Dummy disaggregated graph: short prompts prefill locally, long ones go
    through the prefill queue to the PrefillWorker and back."""
    cp_port, http_port = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=str(tmp_path), DYN_LOG="warning")
    wd = os.path.join(ROOT, "examples", "hello_world", "disagg_skeleton")
    proc = subprocess.Popen([sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "skeleton:Frontend", "-f",
                             "config.yaml", f"--Frontend.port={http_port}", "--control-plane",
                             f"127.0.0.1:{cp_port}"], cwd=wd, env=env, start_new_session=True)
    try:
        def ask(text):
            for _ in range(240):
                try:
                    r = httpx.post(f"http://127.0.0.1:{http_port}/generate", json={"text": text}, timeout=10)
                    if r.status_code == 200:
                        return [l for l in r.text.splitlines() if l]
                except httpx.HTTPError:
                    pass
                time.sleep(0.5)
            raise AssertionError("graph did not come up")

        short = ask("one two three")
        assert short[0] == "<local prefill 3>" and short[1:] == ["three", "two", "one"]
        long = ask(" ".join(f"w{i}" for i in range(12)))
        assert long[0] == "<prefilled 12>" and long[1] == "w11" and len(long) == 13
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)


def _data_url(seed):
    import base64
    import io

    import numpy as np
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(np.random.RandomState(seed).randint(0, 255, (64, 64, 3), dtype=np.uint8)).save(buf, "PNG")
    return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()


@pytest.mark.slow
def test_e2e_multimodal_graph_cpu(tmp_path):
    """LLaVA-style graph on CPU with the tiny-llava preset: image parts are
    encoded by the EncodeWorker component and spliced into the prompt."""
    cp_port, http_port = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=str(tmp_path), DYN_LOG="warning")
    args = [sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "graphs.multimodal_agg:Frontend", "-f",
            "configs/multimodal_agg.yaml", f"--Frontend.port={http_port}", "--Frontend.served_model_name=tiny-llava",
            "--Common.model=tiny-llava", "--Common.block-size=16", "--Common.max-model-len=1024",
            "--Worker.num-gpu-blocks=300", "--Worker.ServiceArgs.resources.gpu=0",
            "--EncodeWorker.ServiceArgs.resources.gpu=0", "--control-plane", f"127.0.0.1:{cp_port}"]
    proc = subprocess.Popen(args, cwd=os.path.join(ROOT, "examples", "llm"), env=env, start_new_session=True)

    def ask(seed):
        body = {"model": "tiny-llava", "max_tokens": 5, "nvext": {"ignore_eos": True}, "temperature": 0,
                "messages": [{"role": "user", "content": [{"type": "text", "text": "what is this?"},
                                                          {"type": "image_url", "image_url": {"url": _data_url(seed)}}]}]}
        for _ in range(300):
            try:
                r = httpx.post(f"http://127.0.0.1:{http_port}/v1/chat/completions", json=body, timeout=60)
                if r.status_code == 200:
                    return r.json()
            except httpx.HTTPError:
                pass
            time.sleep(0.5)
        raise AssertionError("multimodal graph did not serve")

    try:
        a = ask(1)
        assert a["choices"][0]["finish_reason"] == "length"
        assert ask(1)["choices"][0]["message"] == a["choices"][0]["message"]
        st = json.load(open(tmp_path / "dynamo.json"))
        assert "dynamo_EncodeWorker" in st["watchers"]
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)


def test_supervisor_gives_each_worker_process_its_own_gpus(monkeypatch):
    """workers: N with gpu: k -> process i sees GPUs [i*k, (i+1)*k); processes
    sharing one GPU get GPU_MAX_HW_QUEUES=2 (queue time-slicing stalls)."""
    from dynamo_exp_amd.sdk.allocator import ResourceAllocator
    from dynamo_exp_amd.sdk.serve import Supervisor

    monkeypatch.delenv("DYN_DISABLE_AUTO_GPU_ALLOCATION", raising=False)
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    alloc = ResourceAllocator.__new__(ResourceAllocator)
    alloc.gpus = list(range(8))
    alloc.used = {g: 0.0 for g in alloc.gpus}
    sup = Supervisor("ns", "graph:Svc", {}, "127.0.0.1:1", allocator=alloc)
    spawned = []
    monkeypatch.setattr(sup, "_spawn", lambda w, slot: spawned.append((w.name, slot, w.slot_envs[slot])))
    monkeypatch.setattr(sup, "_save", lambda: None)
    sup.add_watcher("ns_W", "W", numprocesses=2, gpus_per_worker=2)
    sup.add_watcher("ns_P", "P", numprocesses=2, gpus_per_worker=0.5)
    envs = {(n, s): e for n, s, e in spawned}
    assert envs[("ns_W", 0)]["HIP_VISIBLE_DEVICES"] == "0,1"
    assert envs[("ns_W", 1)]["HIP_VISIBLE_DEVICES"] == "2,3"
    assert "GPU_MAX_HW_QUEUES" not in envs[("ns_W", 0)]
    assert envs[("ns_P", 0)]["HIP_VISIBLE_DEVICES"] == envs[("ns_P", 1)]["HIP_VISIBLE_DEVICES"] == "4"
    assert envs[("ns_P", 0)]["GPU_MAX_HW_QUEUES"] == "2"
    # a planner scale-up without an explicit share gets the service's configured one (a fractional share
    # here, which a 1-GPU request would not find), an explicit share wins
    sup.service_gpus = {"P": 0.25, "W": 1.0}
    assert sup.gpus_for_add({"service": "P"}) == 0.25
    assert sup.gpus_for_add({"service": "P", "gpus": 1}) == 1.0
    assert sup.gpus_for_add({"service": "X"}) == 0.0


def test_dry_run_places_reference_4p1d_layout():
    """the reference's benchmark layout (4 x PrefillWorker
    TP1 + 1 x Worker TP4, fp8, examples/llm/benchmarks/disagg.yaml:38-58)
    resolves to the 8 GPUs of one node, one HIP_VISIBLE_DEVICES set per worker
    process, and the prefill workers get gpu-memory-utilization 0.9 (not their
    0.5 role default) so a TP1 70B prefill engine fits."""
    from dynamo_exp_amd.llm.workers import parse_worker_args, role_value
    from dynamo_exp_amd.sdk.config import ServiceConfig

    out = subprocess.run([sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "graphs.disagg:Frontend", "-f",
                          "configs/disagg_70b_4p1d.yaml", "--dry-run"],
                         cwd=os.path.join(ROOT, "examples", "llm"), capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, PYTHONPATH=ROOT, DX_NUM_GPUS="8"))
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    place = {p["service"]: p for p in d["placement"]}
    pw, w = place["PrefillWorker"], place["Worker"]
    assert pw["workers"] == 4 and pw["gpus_per_worker"] == 1 and w["workers"] == 1 and w["gpus_per_worker"] == 4
    pre = [s["HIP_VISIBLE_DEVICES"] for s in pw["slots"]]
    dec = w["slots"][0]["HIP_VISIBLE_DEVICES"].split(",")
    assert all("," not in g for g in pre) and len(dec) == 4
    assert sorted(int(g) for g in pre + dec) == list(range(8))  # every GPU once
    assert all(not s for s in place["Frontend"]["slots"])  # CPU-only services get no device
    cfg = ServiceConfig(d["config"])
    pa = parse_worker_args(cfg.as_args("PrefillWorker"))
    da = parse_worker_args(cfg.as_args("Worker"))
    assert pa.quantization == "fp8" and pa.kv_cache_dtype == "fp8" and pa.tensor_parallel_size == 1
    assert role_value(pa, "gpu_memory_utilization", True) == 0.9
    assert role_value(pa, "max_num_seqs", True) == 32  # not given: the prefill role default
    assert da.tensor_parallel_size == 4 and da.remote_prefill and not da.conditional_disagg
    assert role_value(da, "gpu_memory_utilization", False) == 0.95
    # a prefill worker without the flag keeps its role default
    assert role_value(parse_worker_args([]), "gpu_memory_utilization", True) == 0.5
