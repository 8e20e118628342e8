"""Remote-prefill work queue over the control plane's durable queue (the
reference's NATS JetStream `PrefillQueue`, examples/llm/utils/prefill_queue.py
and nats_queue.py): enqueue by decode workers, pull + ack by any prefill
worker, `size()` = messages not yet delivered (consumer num_pending)."""
from __future__ import annotations

import msgpack
from pydantic import BaseModel, Field


class RemotePrefillRequest(BaseModel):
    """reference Patch:4175-4262 RemotePrefillRequest."""

    engine_id: str  # decode worker identity (e.g. its RCCL rank or lease id)
    request_id: str
    prompt_token_ids: list[int]
    sampling_params: dict = Field(default_factory=dict)
    block_ids: list[int] = Field(default_factory=list)  # decode-side blocks (for IPC-write transports)
    computed_block_ids: list[int] = Field(default_factory=list)  # decode-side prefix-cache hits (skip)
    engine_tp: int = 0  # decode engine's TP size (0: look it up in its transfer metadata)
    skip_blocks: int = 0


class PrefillQueue:
    def __init__(self, cp, name: str = "prefill_queue"):
        self.cp = cp
        self.name = name

    @staticmethod
    def encode(req: RemotePrefillRequest) -> bytes:
        return msgpack.packb(req.model_dump(), use_bin_type=True)

    @staticmethod
    def decode(data: bytes) -> RemotePrefillRequest:
        return RemotePrefillRequest(**msgpack.unpackb(data, raw=False))

    async def enqueue(self, req: RemotePrefillRequest) -> int:
        return await self.cp.q_push(self.name, self.encode(req))

    async def dequeue(self, timeout: float = 1.0):
        m = await self.cp.q_pop(self.name, timeout=timeout)
        if m is None:
            return None
        await self.cp.q_ack(self.name, m["seq"])
        return self.decode(m["data"])

    async def size(self) -> int:
        return await self.cp.q_size(self.name)
