"""Disaggregated-serving skeleton with dummy engines (no GPU, no model):
the control flow of examples/llm's disagg graph in ~150 lines.

  Frontend (/generate) -> Processor (tokenize, ask Router) -> Router (least-loaded worker)
     -> DummyWorker.generate: short prompt  -> local "prefill"
                              long prompt   -> RemotePrefillRequest on the prefill queue,
                                               wait for the prefill worker's notification
     <- PrefillWorker: pulls the queue, "computes" the KV, notifies the owning decode worker

    python -m dynamo_exp_amd.sdk.serve skeleton:Frontend -f config.yaml --working-dir examples/hello_world/disagg_skeleton
    curl -X POST localhost:8010/generate -d '{"text": "a long prompt with many many words in it"}'
"""
import asyncio
import logging

from fastapi import FastAPI
from pydantic import BaseModel

from dynamo_exp_amd.disagg.prefill_queue import PrefillQueue, RemotePrefillRequest
from dynamo_exp_amd.sdk import ServiceConfig, async_on_start, depends, dynamo_endpoint, service

log = logging.getLogger("skeleton")
NS = "dynamo-demo"
QUEUE = "dummy_prefill_queue"


class TextRequest(BaseModel):
    text: str


def _cfg(name: str) -> dict:
    return ServiceConfig.get_instance().get(name, {})


@service(dynamo={"namespace": NS})
class PrefillWorker:
    @async_on_start
    async def async_init(self):
        drt = self.__dynamo_runtime__
        self.queue = PrefillQueue(drt.cp, QUEUE)
        self.ns = drt.namespace(NS)
        self.task = asyncio.create_task(self._loop())

    async def _loop(self):
        while True:
            req = await self.queue.dequeue(timeout=1.0)
            if req is None:
                continue
            await asyncio.sleep(0.01 * len(req.prompt_token_ids) / 8)  # "compute" the KV
            await self.ns.publish(f"prefill_done.{req.engine_id}",
                                  {"request_id": req.request_id, "first_token": f"<prefilled {len(req.prompt_token_ids)}>"})

    @dynamo_endpoint()
    async def mock(self, request: dict):
        yield {"ok": True}


@service(dynamo={"namespace": NS}, workers=2)
class DummyWorker:
    prefill = depends(PrefillWorker)  # graph edge: the prefill pool is served with the decode pool

    @async_on_start
    async def async_init(self):
        drt = self.__dynamo_runtime__
        self.engine_id = f"{drt.primary_lease.id:x}"
        self.max_local = int(_cfg("DummyWorker").get("max-local-prefill-length", 8))
        self.queue = PrefillQueue(drt.cp, QUEUE)
        self.pending: dict[str, asyncio.Future] = {}
        sub = await drt.namespace(NS).subscribe(f"prefill_done.{self.engine_id}")

        async def notifications():
            async for m in sub:
                fut = self.pending.pop(m["request_id"], None)
                if fut is not None and not fut.done():
                    fut.set_result(m["first_token"])

        self.task = asyncio.create_task(notifications())

    @dynamo_endpoint()
    async def generate(self, request: dict):
        tokens, rid = request["tokens"], request["request_id"]
        if len(tokens) > self.max_local:
            fut = asyncio.get_running_loop().create_future()
            self.pending[rid] = fut
            await self.queue.enqueue(RemotePrefillRequest(engine_id=self.engine_id, request_id=rid,
                                                          prompt_token_ids=list(range(len(tokens))), block_ids=[]))
            first = await asyncio.wait_for(fut, 30)
        else:
            first = f"<local prefill {len(tokens)}>"
        yield {"worker": self.engine_id, "token": first}
        for t in reversed(tokens):  # "decode"
            yield {"worker": self.engine_id, "token": t}


@service(dynamo={"namespace": NS})
class Router:
    worker = depends(DummyWorker)

    def __init__(self):
        self.load: dict[int, int] = {}

    @dynamo_endpoint()
    async def generate(self, request: dict):
        drt = self.__dynamo_runtime__
        client = await drt.namespace(NS).component("DummyWorker").endpoint("generate").client()
        ids = await client.wait_for_instances(timeout=60)
        wid = min(ids, key=lambda i: self.load.get(i, 0))
        self.load[wid] = self.load.get(wid, 0) + 1
        yield {"worker_id": wid}


@service(dynamo={"namespace": NS})
class Processor:
    worker = depends(DummyWorker)
    router = depends(Router)

    def __init__(self):
        self.n = 0

    @dynamo_endpoint()
    async def generate(self, req: TextRequest):
        self.n += 1
        tokens = req.text.split()
        wid = None
        async for r in self.router.generate({"tokens": tokens}):
            wid = r["worker_id"]
        async for out in self.worker.generate({"tokens": tokens, "request_id": f"req-{self.n}"}, instance_id=wid):
            yield out["token"]


app = FastAPI(title="disagg skeleton")


@service(dynamo={"namespace": NS}, app=app)
class Frontend:
    processor = depends(Processor)

    @dynamo_endpoint(is_api=True)
    async def generate(self, request: TextRequest):
        async for tok in self.processor.generate(request.model_dump_json()):
            yield tok

