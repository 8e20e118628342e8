"""Processor component (reference examples/llm/components/processor.py):
OpenAI request -> chat template + tokenize -> route (random | round-robin |
kv | kv-load via the Router component; the mode is live, watched from the
control plane key `dynamo/processor/router`) -> Worker -> detokenize/stop ->
OpenAI chunks."""
import json

from dynamo_exp_amd.llm.backend import Backend
from dynamo_exp_amd.llm.model_card import ModelDeploymentCard
from dynamo_exp_amd.llm.protocols import ChatCompletionRequest, CompletionRequest
from dynamo_exp_amd.sdk import ServiceConfig, async_on_start, depends, dynamo_endpoint, service

from components.kv_router import Router
from components.worker import Worker

MODE_KEY = "dynamo/processor/router"


def _norm(v) -> str:
    return (v.decode() if isinstance(v, bytes) else str(v)).replace("-", "_")


@service(dynamo={"namespace": "dynamo"})
class Processor:
    worker = depends(Worker)
    router = depends(Router)

    @async_on_start
    async def async_init(self):
        from dynamo_exp_amd.cli.run import make_preprocessor

        cfg = ServiceConfig.get_instance()
        pc = cfg.get("Processor", {})
        model = pc.get("model") or cfg.get("Common", {}).get("model", "llama3-8b")
        self.block_size = int(pc.get("block-size", cfg.get("Common", {}).get("block-size", 64)))
        self.mode = pc.get("router", "round-robin").replace("-", "_")
        self.card = ModelDeploymentCard.load(model, pc.get("served-model-name"), self.block_size)
        self.pre = make_preprocessor(self.card)
        self.backend = Backend(self.pre.tok)
        self.cp = self.__dynamo_runtime__.cp
        await self._watch_mode()

    async def _watch_mode(self):
        """Keep the routing mode live from the control-plane key
        `dynamo/processor/router` through one watch (no per-request get)."""
        import asyncio

        st = await self.cp.watch_prefix(MODE_KEY)
        snap = await st.__anext__()
        for k, v, _ in snap["items"]:
            if k == MODE_KEY:
                self.mode = _norm(v)

        async def pump():
            async for ev in st:
                if ev.get("key") != MODE_KEY:
                    continue
                if ev["type"] == "put":
                    self.mode = _norm(ev["value"])
                elif ev["type"] == "delete":
                    self.mode = self.default_mode

        self.default_mode = self.mode
        self._mode_task = asyncio.create_task(pump())

    async def _route(self, request: dict, ctx):
        mode = self.mode  # one read per request: a live change applies to the next request
        wid = None
        if mode in ("kv", "kv_load"):
            async for d in self.router.generate({"tokens": request["token_ids"], "mode": mode}):
                wid = d["worker_id"]
                request["estimated_prefix_hit_num_blocks"] = d.get("overlap_blocks", 0)
        if wid is not None:
            stream = self.worker.generate(request, ctx, instance_id=wid)
        else:  # random / round_robin, or kv_load before any worker published metrics
            stream = self.worker.generate(request, ctx, mode="round_robin" if mode == "round_robin" else "random")
        async for out in stream:
            yield out

    @dynamo_endpoint()
    async def chat_completions(self, request: dict, context=None):
        req = ChatCompletionRequest(**request)
        pre, ann = self.pre.preprocess_chat(req)
        d = pre.model_dump()
        d["request_id"] = context.id if context else None
        stream = self.backend.generate(d, context, self._route)
        async for ch in self.pre.chat_stream(req, stream, ann):
            yield ch

    @dynamo_endpoint()
    async def completions(self, request: dict, context=None):
        req = CompletionRequest(**request)
        pre, ann = self.pre.preprocess_completion(req)
        d = pre.model_dump()
        stream = self.backend.generate(d, context, self._route)
        async for ch in self.pre.completion_stream(req, stream, ann):
            yield ch
