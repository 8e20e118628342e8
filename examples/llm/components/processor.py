"""Processor component (reference examples/llm/components/processor.py):
OpenAI request -> chat template + tokenize -> route (random | round-robin | kv
via the Router component, mode live in the control plane key
`dynamo/processor/router`) -> Worker -> detokenize/stop -> OpenAI chunks."""
import json

from dynamo_exp_amd.llm.backend import Backend
from dynamo_exp_amd.llm.model_card import ModelDeploymentCard
from dynamo_exp_amd.llm.protocols import ChatCompletionRequest, CompletionRequest
from dynamo_exp_amd.sdk import ServiceConfig, async_on_start, depends, dynamo_endpoint, service

from components.kv_router import Router
from components.worker import Worker


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

    async def _route(self, request: dict, ctx):
        raw = await self.cp.get("dynamo/processor/router")
        mode = raw.decode() if raw else self.mode
        if mode in ("kv", "kv_load"):
            async for d in self.router.generate({"tokens": request["token_ids"]}):
                wid, ov = d["worker_id"], d["overlap_blocks"]
            request["estimated_prefix_hit_num_blocks"] = ov
            stream = self.worker.generate(request, ctx, instance_id=wid)
        else:
            self.worker.mode = "random" if mode == "random" else "round_robin"
            stream = self.worker.generate(request, ctx)
        async for out in stream:
            yield out

    def _engine(self):
        proc = self

        class _E:
            async def generate(self, request, ctx):
                async for out in proc._route(request, ctx):
                    yield out

        return _E()

    @dynamo_endpoint()
    async def chat_completions(self, request: dict, context=None):
        req = ChatCompletionRequest(**request)
        pre, ann = self.pre.preprocess_chat(req)
        d = pre.model_dump()
        d["request_id"] = context.id if context else None
        stream = self.backend.generate(d, context, self._engine().generate)
        async for ch in self.pre.chat_stream(req, stream, ann):
            yield ch

    @dynamo_endpoint()
    async def completions(self, request: dict, context=None):
        req = CompletionRequest(**request)
        pre, ann = self.pre.preprocess_completion(req)
        d = pre.model_dump()
        stream = self.backend.generate(d, context, self._engine().generate)
        async for ch in self.pre.completion_stream(req, stream, ann):
            yield ch
