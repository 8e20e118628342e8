"""Conditional disaggregation policy.

remote prefill iff   prompt_len - prefix_hit_len > max_local_prefill_length
                 and prefill_queue_size < max_prefill_queue_size

(reference examples/llm/components/disagg_router.py:24-66 and the Rust
DisaggregatedRouter lib/llm/src/disagg_router.rs:242-250).  Thresholds are
live-updatable through the control plane key-value store, like the
reference's etcd keys `/dynamo/disagg_router/...` and
`public/components/disagg_router/models/chat/{model}`.
"""
from __future__ import annotations

import asyncio
import json
import logging

log = logging.getLogger("dynamo_exp_amd.disagg")

CONFIG_PREFIX = "dynamo/disagg_router/"


class DisaggregatedRouter:
    def __init__(self, max_local_prefill_length: int = 1000, max_prefill_queue_size: int = 2,
                 model: str | None = None, enabled: bool = True):
        self.max_local_prefill_length = max_local_prefill_length
        self.max_prefill_queue_size = max_prefill_queue_size
        self.model = model
        self.enabled = enabled
        self._watch_task = None

    def prefill_remote(self, prompt_len: int, prefix_hit_len: int = 0, queue_size: int = 0) -> bool:
        if not self.enabled:
            return False
        return (prompt_len - prefix_hit_len) > self.max_local_prefill_length and \
            queue_size < self.max_prefill_queue_size

    def update(self, cfg: dict) -> None:
        if "max_local_prefill_length" in cfg:
            self.max_local_prefill_length = int(cfg["max_local_prefill_length"])
        if "max_prefill_queue_size" in cfg:
            self.max_prefill_queue_size = int(cfg["max_prefill_queue_size"])
        if "enabled" in cfg:
            self.enabled = bool(cfg["enabled"])

    def config_key(self) -> str:
        return CONFIG_PREFIX + (self.model or "default")

    async def watch(self, cp) -> None:
        """Apply live config changes from the control plane."""
        st = await cp.watch_prefix(self.config_key())
        snap = await st.__anext__()
        for _, v, _ in snap["items"]:
            self.update(json.loads(v))

        async def loop():
            async for ev in st:
                if ev["type"] == "put":
                    try:
                        self.update(json.loads(ev["value"]))
                        log.info("disagg router config updated: local<=%d queue<%d", self.max_local_prefill_length,
                                 self.max_prefill_queue_size)
                    except Exception:
                        log.exception("bad disagg config")

        self._watch_task = asyncio.create_task(loop())

    @staticmethod
    async def publish_config(cp, model: str | None, **cfg) -> None:
        await cp.put(CONFIG_PREFIX + (model or "default"), json.dumps(cfg).encode())
