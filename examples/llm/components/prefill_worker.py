"""Prefill worker component (reference examples/llm/components/prefill_worker.py):
pulls RemotePrefillRequests from the prefill queue, ships KV over RCCL."""
import asyncio

from dynamo_exp_amd.llm.workers import PrefillWorker as _Core
from dynamo_exp_amd.llm.workers import parse_worker_args
from dynamo_exp_amd.sdk import ServiceConfig, async_on_shutdown, async_on_start, dynamo_endpoint, service


@service(dynamo={"namespace": "dynamo", "custom_lease": {"ttl": 1}}, resources={"gpu": 1})
class PrefillWorker:
    @async_on_start
    async def async_init(self):
        args = parse_worker_args(ServiceConfig.get_instance().as_args("PrefillWorker"))
        self.core = await _Core(args, self.__dynamo_runtime__, self.__dynamo_component__,
                                self.__dynamo_lease__, "dynamo").start()
        self.task = asyncio.create_task(self.core.run())

    @async_on_shutdown
    async def shutdown(self):
        # lease revoked (planner scale-down): run() stops pulling the queue and
        # returns once everything it dequeued is prefilled and shipped
        lease = self.__dynamo_lease__
        if lease is not None and not lease.is_valid():
            try:
                await asyncio.wait_for(asyncio.shield(self.task), 120)
            except Exception:
                pass
        self.core.shutdown()

    @dynamo_endpoint()
    async def mock(self, request: dict):
        """Health + load endpoint (prefill work arrives through the queue): the
        planner reads `busy` (device-busy fraction over the last second) and
        `dequeued` (prompts pulled so far: the rate policy's arrival estimate)."""
        yield {"inflight": self.core.inflight, "busy": self.core.busy, "dequeued": self.core.dequeued}
