"""Frontend component (reference examples/llm/components/frontend.py): OpenAI
HTTP server; the served model forwards to Processor.chat_completions /
Processor.completions (registered like `llmctl http add chat-models ...`)."""
import asyncio

from dynamo_exp_amd.llm.http_service import HttpService
from dynamo_exp_amd.llm.pipeline import ChatForwarder
from dynamo_exp_amd.sdk import ServiceConfig, async_on_start, depends, dynamo_endpoint, service

from components.processor import Processor


@service(dynamo={"namespace": "dynamo"})
class Frontend:
    processor = depends(Processor)

    @async_on_start
    async def async_init(self):
        cfg = ServiceConfig.get_instance().get("Frontend", {})
        name = cfg.get("served_model_name") or cfg.get("served-model-name") or "llama3-8b"
        port = int(cfg.get("port", 8000))
        drt = self.__dynamo_runtime__
        comp = drt.namespace("dynamo").component("Processor")
        chat = await comp.endpoint("chat_completions").client()
        cmpl = await comp.endpoint("completions").client()
        # SO_REUSEPORT: Frontend.ServiceArgs.workers > 1 runs several frontend
        # processes on the one port (tools/frontend_scale.py)
        self.http = HttpService(port=port, reuse_port=True)
        self.http.manager.add_chat_model(name, ChatForwarder(chat))
        self.http.manager.add_completion_model(name, _Completions(cmpl))
        self.task = asyncio.create_task(self.http.run())

    @dynamo_endpoint()
    async def health(self, request: dict):
        yield {"models": self.http.manager.models()}


class _Completions(ChatForwarder):
    async def completion(self, req, ctx):
        async for ch in self.router.generate(req.model_dump(exclude_none=True), ctx):
            yield ch
