"""KV-aware Router component (reference examples/llm/components/kv_router.py):
`generate({tokens, mode})` -> {worker_id, prefix_hit_rate}; modes kv and
kv_load (kv_router.py:226-245)."""
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
        """mode "kv" (default): prefix overlap + load cost; "kv_load": least
        KV-cache usage only (worker_id None = no metrics yet, caller routes
        randomly)."""
        tokens = request["tokens"]
        ids = self.client.instance_ids()
        if not ids:
            await self.client.wait_for_instances(timeout=60)
            ids = self.client.instance_ids()
        if request.get("mode") == "kv_load":
            wid, usage = self.kv.schedule_least_kv_load(ids)
            yield {"worker_id": wid, "kv_usage": usage, "prefix_hit_rate": 0.0, "overlap_blocks": 0}
            return
        wid, overlap = await self.kv.schedule(tokens, ids)
        isl_blocks = max(1, (len(tokens) + self.block_size - 1) // self.block_size)
        yield {"worker_id": wid, "prefix_hit_rate": overlap / isl_blocks, "overlap_blocks": overlap}
