"""KV-aware Router component (reference examples/llm/components/kv_router.py):
`generate({tokens})` -> {worker_id, prefix_hit_rate}."""
from dynamo_exp_amd.llm.kv_router import KvRouter
from dynamo_exp_amd.sdk import ServiceConfig, async_on_start, depends, dynamo_endpoint, service

from components.worker import Worker


@service(dynamo={"namespace": "dynamo"})
class Router:
    worker = depends(Worker)

    @async_on_start
    async def async_init(self):
        cfg = ServiceConfig.get_instance().get("Router", {})
        self.block_size = int(cfg.get("block-size", 64))
        drt = self.__dynamo_runtime__
        comp = drt.namespace("dynamo").component("Worker")
        self.kv = await KvRouter(comp, self.block_size).start()
        self.client = await comp.endpoint("generate").client()

    @dynamo_endpoint()
    async def generate(self, request: dict):
        tokens = request["tokens"]
        ids = self.client.instance_ids()
        if not ids:
            await self.client.wait_for_instances(timeout=60)
            ids = self.client.instance_ids()
        wid, overlap = await self.kv.schedule(tokens, ids)
        isl_blocks = max(1, (len(tokens) + self.block_size - 1) // self.block_size)
        yield {"worker_id": wid, "prefix_hit_rate": overlap / isl_blocks, "overlap_blocks": overlap}
