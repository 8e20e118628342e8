"""LLM layer on CPU: tokenizer/detok, stop jail, chat template, HTTP frontend
(echo + native engine), and the full distributed path (control plane ->
worker endpoint with the native engine -> frontend model discovery -> HTTP),
with round-robin and KV-aware routing."""
import asyncio
import json

import httpx
import pytest

from dynamo_exp_amd.llm.backend import Backend, StopJail
from dynamo_exp_amd.llm.engines import EchoEngineCore, EchoEngineFull, NativeEngine
from dynamo_exp_amd.llm.http_service import HttpService, RequestTemplate
from dynamo_exp_amd.llm.pipeline import FullPipeline, LocalPipeline
from dynamo_exp_amd.llm.preprocessor import OpenAIPreprocessor, PromptFormatter
from dynamo_exp_amd.llm.tokenizer import SyntheticTokenizer


def run(coro, t=60):
    return asyncio.run(asyncio.wait_for(coro, t))


def test_synthetic_tokenizer_and_decode_stream():
    tok = SyntheticTokenizer(512, 0, [1])
    ids = tok.encode("héllo wörld <|eot_id|>!")
    assert tok.decode(ids, skip_special_tokens=False) == "héllo wörld <|eot_id|>!"
    ds = tok.decode_stream([])
    text = "".join(p for t in tok.encode("a longer multi-byte ✓ string" * 5) if (p := ds.step(t)))
    assert text == "a longer multi-byte ✓ string" * 5


def test_stop_jail():
    j = StopJail(["STOP", "</s>"])
    out, m = j.push("hello ST")
    assert out == "hello " and not m
    out, m = j.push("OP world")
    assert out == "" and m
    j2 = StopJail(["xyz"])
    assert j2.push("abx") == ("ab", False)
    assert j2.push("q") == ("xq", False)


def test_chat_template_llama3():
    fmt = PromptFormatter(None, "<|begin_of_text|>", "<|end_of_text|>", ["llama3_date_time"])
    s = fmt.render([{"role": "system", "content": "sys"}, {"role": "user", "content": "hi"}])
    assert s.startswith("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\nsys<|eot_id|>")
    assert s.endswith("<|start_header_id|>assistant<|end_header_id|>\n\n")


def _echo_service():
    tok = SyntheticTokenizer(1024, 0, [1])
    pre = OpenAIPreprocessor("echo", tok, eos_token_ids=[1])
    svc = HttpService(request_template=RequestTemplate(model="echo", max_completion_tokens=64))
    svc.manager.add_chat_model("echo", LocalPipeline(pre, Backend(tok), EchoEngineCore()))
    svc.manager.add_completion_model("echo", LocalPipeline(pre, Backend(tok), EchoEngineCore()))
    svc.manager.add_chat_model("echo_full", FullPipeline(EchoEngineFull()))
    return svc


def test_http_echo(monkeypatch):
    monkeypatch.setenv("DYN_TOKEN_ECHO_DELAY_MS", "0")
    svc = _echo_service()

    async def main():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=svc.app), base_url="http://t") as c:
            r = await c.get("/v1/models")
            assert {m["id"] for m in r.json()["data"]} == {"echo", "echo_full"}
            # unary, request template fills the model
            r = await c.post("/v1/completions", json={"prompt": "hello world", "max_tokens": 100})
            assert r.status_code == 200, r.text
            assert r.json()["choices"][0]["text"] == "hello world"
            # streaming chat through the token-level echo (echoes the templated prompt)
            r = await c.post("/v1/chat/completions", json={"model": "echo", "stream": True,
                                                           "messages": [{"role": "user", "content": "ping"}]})
            lines = [l for l in r.text.split("\n") if l.startswith("data: ")]
            assert lines[-1] == "data: [DONE]"
            text = "".join(json.loads(l[6:])["choices"][0]["delta"].get("content") or "" for l in lines[:-1])
            assert "ping" in text
            # stop strings cut the output
            r = await c.post("/v1/completions", json={"model": "echo", "prompt": "abc STOP def", "stop": ["STOP"]})
            assert r.json()["choices"][0]["text"] == "abc "
            assert r.json()["choices"][0]["finish_reason"] == "stop"
            r = await c.post("/v1/chat/completions", json={"model": "echo_full",
                                                           "messages": [{"role": "user", "content": "xyz"}]})
            assert r.json()["choices"][0]["message"]["content"] == "xyz"
            r = await c.post("/v1/chat/completions", json={"model": "nope", "messages": []})
            assert r.status_code == 404
            m = (await c.get("/metrics")).text
            assert 'dynamo_http_service_requests_total{endpoint="completions",model="echo",request_type="unary",status="success"}' in m
            assert "dynamo_http_service_time_to_first_token_seconds" in m

    run(main())


def _tiny_native():
    from dynamo_exp_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine

    eng = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=1024, num_gpu_blocks=300,
                                 max_num_seqs=8))
    return eng, AsyncLLMEngine(eng).start()


def test_http_native_engine_cpu():
    eng, ae = _tiny_native()
    tok = SyntheticTokenizer(512, 0, [2])
    pre = OpenAIPreprocessor("tiny", tok, eos_token_ids=[2])
    svc = HttpService()
    svc.manager.add_chat_model("tiny", LocalPipeline(pre, Backend(tok), NativeEngine(ae)))

    async def main():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=svc.app), base_url="http://t") as c:
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny", "messages": [{"role": "user", "content": "hello"}], "max_tokens": 7,
                "nvext": {"ignore_eos": True}, "stream_options": {"include_usage": True}, "stream": True})
            lines = [json.loads(l[6:]) for l in r.text.split("\n") if l.startswith("data: {")]
            usage = lines[-1]["usage"]
            assert usage["completion_tokens"] == 7
            assert lines[-2]["choices"][0]["finish_reason"] == "length"

    try:
        run(main())
    finally:
        ae.shutdown()


def test_distributed_worker_frontend_discovery():
    from dynamo_exp_amd.cli.run import make_preprocessor
    from dynamo_exp_amd.llm.discovery import ModelWatcher
    from dynamo_exp_amd.llm.kv_router import KvEventPublisher, KvMetricsPublisher
    from dynamo_exp_amd.llm.model_card import ModelDeploymentCard, attach
    from dynamo_exp_amd.llm.pipeline import core_handler
    from dynamo_exp_amd.runtime import BackgroundServer, DistributedRuntime

    cp = BackgroundServer().start()
    engines = [_tiny_native() for _ in range(2)]

    async def main():
        card = ModelDeploymentCard.load("tiny", "tiny-model", block_size=16)
        workers = []
        for eng, ae in engines:
            drt = await DistributedRuntime.create(cp.address)
            comp = drt.namespace("dx").component("backend")
            ep = comp.endpoint("generate")
            pre = make_preprocessor(card)
            pub = KvEventPublisher(comp, drt.primary_lease.id, 16, asyncio.get_running_loop())
            eng.add_kv_event_listener(pub.on_engine_events)
            mp = await KvMetricsPublisher(comp, drt.primary_lease.id, eng.forward_pass_metrics, 0.05).start()
            await ep.register(core_handler(Backend(pre.tok), NativeEngine(ae)), stats_handler=mp.stats_handler)
            await attach(drt, ep, card, "backend", router_mode="kv")
            workers.append((drt, mp))
        fe = await DistributedRuntime.create(cp.address, is_static=True)
        svc = HttpService()
        watcher = await ModelWatcher(fe, svc.manager).start()
        assert svc.manager.models() == ["tiny-model"]
        pipe = svc.manager.chat["tiny-model"]
        await pipe.router.client.wait_for_instances(timeout=5, n=2)
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=svc.app), base_url="http://t") as c:
            long_msg = "the same long shared system prompt " * 8
            for i in range(4):
                r = await c.post("/v1/chat/completions", json={
                    "model": "tiny-model", "max_tokens": 5, "nvext": {"ignore_eos": True},
                    "messages": [{"role": "system", "content": long_msg}, {"role": "user", "content": f"q{i}"}]})
                assert r.status_code == 200, r.text
                assert r.json()["choices"][0]["finish_reason"] == "length"
                await asyncio.sleep(0.2)  # let KV events reach the indexer
            kv = pipe.router.kv
            assert kv.indexer.events > 0
            # prefix-sharing requests concentrate on one worker (KV-aware)
            hits = [e.kv.prefix_hit_tokens for e, _ in engines]
            assert max(hits) > 0
        # lease revoke removes instances; model disappears when all are gone
        for drt, mp in workers:
            mp.stop()
            await drt.primary_lease.revoke()
        for _ in range(100):
            if not svc.manager.models():
                break
            await asyncio.sleep(0.05)
        assert svc.manager.models() == []
        for drt, _ in workers:
            await drt.close(1)
        await fe.close(1)

    try:
        run(main(), 120)
    finally:
        for _, ae in engines:
            ae.shutdown()
        cp.stop()
