"""Frontend model discovery (reference lib/llm/src/http/service/discovery.rs).

Watches `models/{type}/{name}:{lease}` on the control plane.  For each new
model name it builds a pipeline:
  * `backend` entries: MDC -> tokenizer + prompt formatter -> preprocessor,
    routed to the worker endpoint with the entry's router mode (round_robin,
    random or kv -- the reference hard-codes Random here, §2.16);
  * `chat` / `completion` entries: raw OpenAI forwarding to the endpoint.
A model disappears when its last instance's entry is deleted (lease expiry /
revoke).
"""
from __future__ import annotations

import asyncio
import logging

from ..runtime.distributed import DistributedRuntime
from .backend import Backend
from .http_service import ModelManager
from .kv_router import KvRouter
from .model_card import MODELS_PREFIX, ModelDeploymentCard, ModelEntry
from .pipeline import ChatForwarder, RemotePipeline, WorkerRouter
from .preprocessor import OpenAIPreprocessor, PromptFormatter
from .tokenizer import load_tokenizer

log = logging.getLogger("dynamo_exp_amd.discovery")


async def build_preprocessor(drt: DistributedRuntime, entry: ModelEntry) -> OpenAIPreprocessor:
    card = None
    if entry.mdc_key:
        raw = await drt.cp.get(entry.mdc_key)
        if raw is not None:
            card = ModelDeploymentCard.from_json(raw)
            await card.move_from_blob_store(drt.cp)
    if card is None:
        card = ModelDeploymentCard.load("llama3-8b", entry.name)
    mc = card.model_config()
    tok = load_tokenizer(card.local_dir(), mc.vocab_size, mc.bos_token_id, mc.eos_token_id)
    tmpl = getattr(tok, "chat_template", None)
    fmt = PromptFormatter(tmpl, tok.bos_token, tok.eos_token, card.prompt_context)
    return OpenAIPreprocessor(entry.name, tok, fmt, eos_token_ids=mc.eos_token_id, mdc_sum=card.mdcsum(),
                              context_length=card.context_length)


class ModelWatcher:
    def __init__(self, drt: DistributedRuntime, manager: ModelManager, router_mode: str | None = None,
                 prefix: str = MODELS_PREFIX):
        self.drt, self.manager = drt, manager
        self.prefix = prefix
        self.router_mode = router_mode  # override entry.router_mode if set
        # (model_type, name) -> live entry keys; a chat and a completion entry of
        # one name (llmctl) are independent, a backend entry serves both
        self.instances: dict[tuple[str, str], set[str]] = {}
        self.clients = {}
        self._task = None
        self.ready = asyncio.Event()

    async def start(self) -> "ModelWatcher":
        st = await self.drt.cp.watch_prefix(self.prefix)
        snap = await st.__anext__()
        for k, v, _ in snap["items"]:
            await self._put(k, v)
        self.ready.set()

        async def loop():
            async for ev in st:
                try:
                    if ev["type"] == "put":
                        await self._put(ev["key"], ev["value"])
                    else:
                        await self._delete(ev["key"])
                except Exception:
                    log.exception("model watcher event failed")

        self._task = asyncio.create_task(loop())
        return self

    async def _put(self, key: str, value: bytes) -> None:
        entry = ModelEntry.from_json(value)
        ident = (entry.model_type, entry.name)
        inst = self.instances.setdefault(ident, set())
        first = not inst
        inst.add(key)
        if not first:
            return
        ns, comp, ep = entry.endpoint.replace(".", "/").split("/")
        endpoint = self.drt.namespace(ns).component(comp).endpoint(ep)
        client = await endpoint.client()
        self.clients[ident] = client
        mode = self.router_mode or entry.router_mode
        if entry.model_type == "backend":
            pre = await build_preprocessor(self.drt, entry)
            kv = None
            if mode == "kv":
                kv = await KvRouter(self.drt.namespace(ns).component(comp), entry.kv_block_size).start()
            pipe = RemotePipeline(pre, WorkerRouter(client, mode, kv))
            self.manager.add_chat_model(entry.name, pipe)
            self.manager.add_completion_model(entry.name, pipe)
        elif entry.model_type == "chat":
            self.manager.add_chat_model(entry.name, ChatForwarder(client, mode))
        else:
            self.manager.add_completion_model(entry.name, ChatForwarder(client, mode))
        log.info("model %s added (%s via %s, router=%s)", entry.name, entry.model_type, entry.endpoint, mode)

    async def _delete(self, key: str) -> None:
        for ident, inst in list(self.instances.items()):
            if key in inst:
                inst.discard(key)
                if not inst:
                    mtype, name = ident
                    if mtype == "chat":
                        self.manager.remove_chat_model(name)
                    elif mtype == "completion":
                        self.manager.remove_completion_model(name)
                    else:
                        self.manager.remove_model(name)
                    c = self.clients.pop(ident, None)
                    if c is not None:
                        await c.close()
                    del self.instances[ident]
                    log.info("model %s (%s) removed", name, mtype)
