"""Prometheus / Grafana deploy assets (reference deploy/metrics/*,
deploy/docker-compose.yml:33-78): every metric a dashboard panel queries is
one this framework exports -- the worker-load exporter (cli/metrics.py), the
OpenAI frontend (llm/http_service.py) or the engine phase / KV-transfer
histograms (utils/tracing.py, served by workers with --metrics-port)."""
import json
import os
import re

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")


def _exported() -> set[str]:
    from prometheus_client import CollectorRegistry

    from dynamo_exp_amd.cli.metrics import PrometheusMetrics
    from dynamo_exp_amd.llm.http_service import Metrics
    from dynamo_exp_amd.utils.tracing import RequestTimer

    names = set()
    for reg in (PrometheusMetrics(CollectorRegistry()).registry, Metrics().registry, RequestTimer().registry):
        for fam in reg.collect():
            names.add(fam.name)
            if fam.type == "counter":
                names.add(fam.name + "_total")
            elif fam.type == "histogram":
                names.update(fam.name + s for s in ("_bucket", "_sum", "_count"))
    return names


def test_dashboard_queries_only_exported_metrics():
    with open(os.path.join(DEPLOY, "metrics", "grafana-dashboard.json")) as f:
        dash = json.load(f)
    exported = _exported()
    used = set()
    panels = [p for p in dash["panels"] if p["type"] != "row"]
    assert len(panels) >= 15
    for p in panels:
        assert p["targets"], p["title"]
        for t in p["targets"]:
            for name in re.findall(r"\b((?:llm|dynamo)_[a-z_]+)\b", t["expr"]):
                assert name in exported, (p["title"], name)
                used.add(name)
    # the panels cover the three sources, TTFT / ITL histograms and KV-transfer bandwidth
    assert any(n.startswith("llm_") for n in used)
    assert "dynamo_http_service_time_to_first_token_seconds_bucket" in used
    assert "dynamo_http_service_inter_token_latency_seconds_bucket" in used
    assert "dynamo_engine_kv_transfer_bytes_total" in used
    for v in dash["templating"]["list"]:
        for name in re.findall(r"\b((?:llm|dynamo)_[a-z_]+)\b", v["query"]):
            assert name in exported


def test_prometheus_and_compose_config():
    with open(os.path.join(DEPLOY, "metrics", "prometheus.yml")) as f:
        prom = yaml.safe_load(f)
    jobs = {j["job_name"]: j for j in prom["scrape_configs"]}
    assert {"dx_worker_load", "dx_frontend", "dx_engines"} <= set(jobs)
    with open(os.path.join(DEPLOY, "docker-compose.yml")) as f:
        compose = yaml.safe_load(f)
    for svc in ("prometheus", "grafana"):
        for vol in compose["services"][svc]["volumes"]:
            src = vol.split(":")[0]
            assert os.path.exists(os.path.join(DEPLOY, src)), src
    with open(os.path.join(DEPLOY, "metrics", "grafana-datasources.yml")) as f:
        ds = yaml.safe_load(f)
    assert ds["datasources"][0]["uid"] == "prometheus"


def test_worker_engine_metrics_port():
    """--metrics-port serves a worker's engine histograms over HTTP."""
    import socket
    import urllib.request

    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams
    from dynamo_exp_amd.llm.workers import _serve_engine_metrics, parse_worker_args
    from dynamo_exp_amd.parallel.tp import ReplicatedEngine

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    eng = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64,
                                 max_num_seqs=2))
    eng.add_request("m", list(range(30, 60)), SamplingParams(max_tokens=3, ignore_eos=True))
    while eng.has_unfinished():
        eng.step()
    _serve_engine_metrics(parse_worker_args(["--metrics-port", str(port)]), ReplicatedEngine(eng, None, 0, 1))
    body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
    assert "dynamo_engine_time_to_first_token_seconds_count 1.0" in body
