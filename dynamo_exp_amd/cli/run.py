"""`run` -- single-binary launcher (reference launch/dynamo-run).

    python -m dynamo_exp_amd.cli.run in=<input> out=<engine> [flags] [-- extra args for py engines]

in:  http | text | stdin | batch:<file.jsonl> | dyn://ns.comp.ep | none
out: native | echo_core | echo_full | sim | pystr:<file.py> | pytok:<file.py> | dyn://ns.comp.ep
     (sim = timing-faithful engine stand-in for frontend benchmarks, engine/sim.py)

Examples
  run in=http out=native --model-path llama3-8b --http-port 8080     # aggregated single process
  run in=dyn://dynamo.backend.generate out=native --model-path llama3-8b   # worker
  run in=http out=dyn://dynamo.backend.generate --router-mode kv            # frontend
  run in=batch:prompts.jsonl out=echo_core                                   # offline batch
Flags mirror launch/dynamo-run/src/flags.rs (--router-mode kv works here; the
reference hits todo!() at flags.rs:247).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import sys
import time

from ..llm.backend import Backend
from ..llm.engines import EchoEngineCore, EchoEngineFull, NativeEngine, PythonStringEngine, PythonTokenEngine
from ..llm.http_service import HttpService, RequestTemplate
from ..llm.model_card import ModelDeploymentCard, attach
from ..llm.pipeline import FullPipeline, LocalPipeline, RemotePipeline, WorkerRouter, core_handler
from ..llm.preprocessor import OpenAIPreprocessor, PromptFormatter, aggregate_chat
from ..llm.protocols import ChatCompletionRequest, ChatMessage
from ..llm.tokenizer import load_tokenizer
from ..runtime import configure_logging
from ..runtime.context import Context

log = logging.getLogger("dynamo_exp_amd.run")


def parse_args(argv: list[str]):
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    inp, out = "text", "native"
    rest = []
    for a in argv:
        if a.startswith("in="):
            inp = a[3:]
        elif a.startswith("out="):
            out = a[4:]
        else:
            rest.append(a)
    ap = argparse.ArgumentParser(prog="run")
    ap.add_argument("--model-path", default=os.environ.get("DX_MODEL", "llama3-8b"))
    ap.add_argument("--model-name", default=None)
    ap.add_argument("--model-config", default=None)
    ap.add_argument("--http-port", type=int, default=8080)
    ap.add_argument("--http-host", default="0.0.0.0")
    ap.add_argument("--tensor-parallel-size", type=int, default=1)
    ap.add_argument("--pipeline-parallel-size", type=int, default=1,
                    help="accepted for CLI parity; only 1 is supported (single-node TP engine)")
    ap.add_argument("--base-gpu-id", type=int, default=0)
    ap.add_argument("--num-nodes", type=int, default=1)
    ap.add_argument("--node-rank", type=int, default=0)
    ap.add_argument("--leader-addr", default=None)
    ap.add_argument("--router-mode", default="round_robin", choices=["random", "round-robin", "round_robin", "kv"])
    ap.add_argument("--kv-cache-block-size", type=int, default=64)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.9)
    ap.add_argument("--extra-engine-args", default=None, help="JSON file or inline JSON merged into EngineConfig")
    ap.add_argument("--request-template", default=None)
    ap.add_argument("--control-plane", default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("-v", action="count", default=0)
    a = ap.parse_args(rest)
    a.input, a.output, a.extra = inp, out, extra
    a.router_mode = a.router_mode.replace("-", "_")
    if a.num_nodes > 1:
        raise SystemExit("multi-node engines are not supported in this version (single 8-GPU node)")
    check_pipeline_parallel(a.pipeline_parallel_size)
    return a


def check_pipeline_parallel(pp: int) -> None:
    """The reference's vLLM 0.8 engine passes one pipeline stage per node
    (lib/engines/vllm0_8/src/lib.rs:378-382); this framework is single-node
    (one node of 8 x 288 GB holds Llama-3-70B at TP <= 8 without pipeline
    stages), so any value other than 1 is refused instead of ignored."""
    if pp != 1:
        raise SystemExit(f"--pipeline-parallel-size {pp}: pipeline parallelism is not supported "
                         "(use --tensor-parallel-size)")


def _card(a) -> ModelDeploymentCard:
    return ModelDeploymentCard.load(a.model_path, a.model_name, a.kv_cache_block_size)


def make_preprocessor(card: ModelDeploymentCard) -> OpenAIPreprocessor:
    mc = card.model_config()
    tok = load_tokenizer(card.local_dir(), mc.vocab_size, mc.bos_token_id, mc.eos_token_id)
    fmt = PromptFormatter(getattr(tok, "chat_template", None), tok.bos_token, tok.eos_token, card.prompt_context)
    pre = OpenAIPreprocessor(card.display_name, tok, fmt, eos_token_ids=mc.eos_token_id, mdc_sum=card.mdcsum(),
                             context_length=card.context_length)
    if mc.vision and mc.image_token_id is not None:
        pre.image_token_id = mc.image_token_id
        pre.image_tokens = (mc.vision["image_size"] // mc.vision["patch_size"]) ** 2
    return pre


def make_native_engine(a):
    from ..engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine

    from ..engine.policy import SERVING_DEFAULTS

    # the benchmarked scheduler policy (engine/policy.py); --extra-engine-args overrides it
    kw = dict(SERVING_DEFAULTS)
    if a.extra_engine_args:
        src = a.extra_engine_args
        kw.update(json.load(open(src)) if os.path.exists(src) else json.loads(src))
    import torch

    dev = f"cuda:{a.base_gpu_id}" if torch.cuda.is_available() else "cpu"
    cfg = EngineConfig.from_args(model=a.model_path, block_size=a.kv_cache_block_size, max_model_len=a.max_model_len,
                                 max_num_seqs=a.max_num_seqs, gpu_memory_utilization=a.gpu_memory_utilization,
                                 use_cuda_graph=not a.no_graph, device=dev, **kw)
    if a.tensor_parallel_size > 1:
        from ..parallel.tp import make_tp_engine

        return make_tp_engine(cfg, a.tensor_parallel_size, a.base_gpu_id)
    eng = LLMEngine(cfg)
    if dev.startswith("cuda"):
        eng.warmup()
    ae = AsyncLLMEngine(eng).start()
    return NativeEngine(ae, eng.eos_token_ids)


def make_engine(a):
    o = a.output
    if o == "echo_core":
        return EchoEngineCore()
    if o == "echo_full":
        return EchoEngineFull()
    if o == "sim":
        from ..engine.engine import AsyncLLMEngine
        from ..engine.sim import SimLLMEngine

        sim = SimLLMEngine(max_num_seqs=a.max_num_seqs)
        return NativeEngine(AsyncLLMEngine(sim).start(), sim.eos_token_ids)
    if o in ("native", "vllm", "sglang"):  # the first-party engine serves every "engine" out=
        return make_native_engine(a)
    if o.startswith("pytok:"):
        return PythonTokenEngine(o[6:], a.extra)
    if o.startswith("pystr:"):
        return PythonStringEngine(o[6:], a.extra)
    raise SystemExit(f"unknown out={o}")


def parse_dyn(url: str) -> tuple[str, str, str]:
    p = url[len("dyn://"):]
    sep = "/" if "/" in p else "."
    ns, comp, ep = p.split(sep)
    return ns, comp, ep


async def _pipeline_for(a, card):
    if a.output.startswith("dyn://"):
        from ..runtime.distributed import DistributedRuntime

        drt = await DistributedRuntime.create(a.control_plane, is_static=True)
        ns, comp, ep = parse_dyn(a.output)
        client = await drt.namespace(ns).component(comp).endpoint(ep).client()
        await client.wait_for_instances(timeout=300)
        kv = None
        if a.router_mode == "kv":
            from ..llm.kv_router import KvRouter

            kv = await KvRouter(drt.namespace(ns).component(comp), a.kv_cache_block_size).start()
        return RemotePipeline(make_preprocessor(card), WorkerRouter(client, a.router_mode, kv)), drt
    eng = make_engine(a)
    if getattr(eng, "kind", "core") == "full":
        return FullPipeline(eng), None
    pre = make_preprocessor(card)
    return LocalPipeline(pre, Backend(pre.tok), eng), None


async def run_http(a):
    card = _card(a)
    pipe, _ = await _pipeline_for(a, card)
    tmpl = RequestTemplate.load(a.request_template) if a.request_template else None
    svc = HttpService(a.http_host, a.http_port, tmpl)
    svc.manager.add_chat_model(card.display_name, pipe)
    svc.manager.add_completion_model(card.display_name, pipe)
    log.info("serving %s on http://%s:%d", card.display_name, a.http_host, a.http_port)
    await svc.run()


async def run_text(a, stream_in=None):
    card = _card(a)
    pipe, _ = await _pipeline_for(a, card)
    history = []
    interactive = stream_in is None and sys.stdin.isatty()
    src = stream_in or sys.stdin
    while True:
        if interactive:
            print("User: ", end="", flush=True)
        line = src.readline()
        if not line:
            break
        line = line.strip()
        if not line:
            continue
        history.append({"role": "user", "content": line})
        req = ChatCompletionRequest(model=card.display_name, messages=[ChatMessage(**m) for m in history],
                                    stream=True, max_tokens=256)
        out = []
        async for ch in pipe.chat(req, Context()):
            for c in ch.get("choices", []):
                t = c.get("delta", {}).get("content")
                if t:
                    out.append(t)
                    print(t, end="", flush=True)
        print()
        history.append({"role": "assistant", "content": "".join(out)})
        if not interactive and stream_in is None:
            history = []


async def run_batch(a, path: str):
    """Reference input/batch.rs: one JSON {"text": ...} per line -> output.jsonl."""
    card = _card(a)
    pipe, _ = await _pipeline_for(a, card)
    outp = os.path.join(os.path.dirname(os.path.abspath(path)), "output.jsonl")
    sem = asyncio.Semaphore(64)
    tok = getattr(getattr(pipe, "pre", None), "tok", None)

    async def one(i, entry):
        async with sem:
            t0 = time.perf_counter()
            req = ChatCompletionRequest(model=card.display_name, messages=[ChatMessage(role="user", content=entry["text"])],
                                        max_tokens=entry.get("max_tokens", 256), stream=True)
            resp = await aggregate_chat(pipe.chat(req, Context()))
            text = resp["choices"][0]["message"]["content"]
            return {"text": entry["text"], "response": text,
                    "tokens_in": len(tok.encode(entry["text"])) if tok else None,
                    "tokens_out": len(tok.encode(text)) if tok else None,
                    "elapsed_ms": round((time.perf_counter() - t0) * 1000, 1)}

    entries = [json.loads(l) for l in open(path) if l.strip()]
    t0 = time.perf_counter()
    results = await asyncio.gather(*[one(i, e) for i, e in enumerate(entries)])
    with open(outp, "w") as f:
        for r in results:
            f.write(json.dumps(r) + "\n")
    log.info("batch: %d prompts in %.2fs -> %s", len(entries), time.perf_counter() - t0, outp)
    return outp


async def run_endpoint(a):
    """Worker: serve Backend+engine on dyn://ns.comp.ep and register the model."""
    from ..runtime.distributed import DistributedRuntime

    drt = await DistributedRuntime.create(a.control_plane)
    ns, comp, ep = parse_dyn(a.input)
    card = _card(a)
    engine = make_engine(a)
    component = drt.namespace(ns).component(comp)
    await component.create_service()
    endpoint = component.endpoint(ep)
    if getattr(engine, "kind", "core") == "full":
        handler = lambda req, ctx: engine.generate(req, ctx)  # noqa: E731
        mtype = "chat"
    else:
        pre = make_preprocessor(card)
        handler = core_handler(Backend(pre.tok), engine)
        mtype = "backend"
    stats = None
    ae = getattr(engine, "ae", None)
    if ae is not None:
        from ..llm.kv_router import KvEventPublisher, KvMetricsPublisher

        wid = drt.primary_lease.id
        pub = KvEventPublisher(component, wid, a.kv_cache_block_size, asyncio.get_running_loop())
        ae.engine.add_kv_event_listener(pub.on_engine_events)
        mp = await KvMetricsPublisher(component, wid, ae.engine.forward_pass_metrics).start()
        stats = mp.stats_handler
    await endpoint.register(handler, stats_handler=stats)
    await attach(drt, endpoint, card, mtype, a.router_mode)
    log.info("worker serving %s at %s (lease %x)", card.display_name, endpoint.path, drt.primary_lease.id)
    await drt.shutdown_event.wait()
    await drt.close()


def main(argv=None):
    a = parse_args(list(sys.argv[1:] if argv is None else argv))
    os.environ.setdefault("DYN_LOG", ["info", "debug", "trace"][min(a.v, 2)])
    configure_logging()
    if a.input == "http":
        asyncio.run(run_http(a))
    elif a.input in ("text",):
        asyncio.run(run_text(a))
    elif a.input == "stdin":
        asyncio.run(run_text(a, sys.stdin))
    elif a.input.startswith("batch:"):
        asyncio.run(run_batch(a, a.input[6:]))
    elif a.input.startswith("dyn://"):
        asyncio.run(run_endpoint(a))
    elif a.input == "none":
        eng = make_engine(a)
        print("engine started; Ctrl-C to exit", flush=True)
        try:
            while True:
                time.sleep(3600)
        except KeyboardInterrupt:
            pass
    else:
        raise SystemExit(f"unknown in={a.input}")


if __name__ == "__main__":
    main()
