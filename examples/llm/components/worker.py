"""Aggregated / decode worker component (reference examples/llm/components/worker.py).

Config keys (YAML section `Worker`, rendered to argv by ServiceConfig.as_args):
  model, block-size, max-model-len, max-num-seqs, remote-prefill, conditional-disagg,
  max-local-prefill-length, max-prefill-queue-size, gpu-memory-utilization
Custom lease TTL 1 s (so the planner can drain it fast).
"""
from dynamo_exp_amd.llm.workers import LLMWorker, parse_worker_args
from dynamo_exp_amd.sdk import ServiceConfig, async_on_shutdown, async_on_start, dynamo_endpoint, service


@service(dynamo={"namespace": "dynamo", "custom_lease": {"ttl": 1}}, resources={"gpu": 1})
class Worker:
    @async_on_start
    async def async_init(self):
        args = parse_worker_args(ServiceConfig.get_instance().as_args("Worker"))
        self.core = await LLMWorker(args, self.__dynamo_runtime__, self.__dynamo_component__,
                                    self.__dynamo_lease__, "dynamo").start()

    @async_on_shutdown
    def shutdown(self):
        self.core.shutdown()

    @dynamo_endpoint()
    async def generate(self, request: dict, context=None):
        async for out in self.core.generate(request, context):
            yield out
