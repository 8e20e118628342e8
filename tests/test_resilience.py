"""Fault injection, retry-before-first-token, request ids and request-phase
metrics (SURVEY §5.1 / §5.3 build targets)."""
import asyncio

import pytest

from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams
from dynamo_exp_amd.llm.pipeline import WorkerRouter
from dynamo_exp_amd.runtime import BackgroundServer, Context, DistributedRuntime, EndpointError
from dynamo_exp_amd.utils import tracing
from dynamo_exp_amd.utils.faults import FaultInjector, InjectedFault


@pytest.fixture(scope="module")
def cp():
    s = BackgroundServer().start()
    yield s.address
    s.stop()


def test_fault_injector_spec_and_hooks():
    f = FaultInjector("endpoint.error_rate=1.0,kv_transfer.delay_ms=1", seed=0)
    with pytest.raises(InjectedFault):
        f.on_request()
    f.disarm("endpoint.error_rate")
    f.on_request()
    f.before_kv_transfer_sync()
    f.arm("kv_transfer.fail_rate", 1.0)
    with pytest.raises(InjectedFault):
        asyncio.run(f.before_kv_transfer())


def test_retry_before_first_token(cp):
    """One of two workers fails every request before producing output: the
    router re-routes, so every request still completes."""

    async def main():
        drts = [await DistributedRuntime.create(cp) for _ in range(2)]
        faulty = FaultInjector("endpoint.error_rate=1.0")

        def handler(i):
            async def h(req, ctx):
                if i == 0:
                    faulty.on_request()
                for t in range(3):
                    yield {"w": i, "t": t}
            return h

        for i, d in enumerate(drts):
            await d.namespace("rs").component("W").endpoint("gen").register(handler(i))
        drt = await DistributedRuntime.create(cp, is_static=True)
        client = await drt.namespace("rs").component("W").endpoint("gen").client()
        await client.wait_for_instances(timeout=10, n=2)
        router = WorkerRouter(client, "round_robin", retries=1)
        for _ in range(4):
            outs = [o async for o in router.generate({"x": 1}, Context())]
            assert [o["w"] for o in outs] == [1, 1, 1]
        no_retry = WorkerRouter(client, "round_robin", retries=0)
        errors = 0
        for _ in range(2):
            try:
                _ = [o async for o in no_retry.generate({"x": 1}, Context())]
            except EndpointError:
                errors += 1
        assert errors == 1
        for d in drts + [drt]:
            await d.close(1)

    asyncio.run(main())


def test_request_timer_histograms():
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64,
                               max_num_seqs=4, seed=3))
    for i in range(3):
        e.add_request(f"r{i}", list(range(10, 40)), SamplingParams(max_tokens=5, ignore_eos=True))
    while e.has_unfinished():
        e.step()
    from prometheus_client import generate_latest

    text = generate_latest(e.request_timer.registry).decode()
    assert 'dynamo_engine_time_to_first_token_seconds_count 3.0' in text
    assert 'dynamo_engine_queue_seconds_count 3.0' in text
    assert 'dynamo_engine_requests_finished_total{reason="length"} 3.0' in text


def test_roctx_spans_are_noops_without_env(monkeypatch):
    with tracing.span("x"):
        pass
    tracing.mark("m")
