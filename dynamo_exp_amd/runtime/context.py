"""Request context with graceful stop vs. hard kill (reference
lib/runtime/src/engine.rs:47 AsyncEngineContext, pipeline/context.rs:33)."""
from __future__ import annotations

import asyncio
import uuid


class Context:
    __slots__ = ("id", "_stopped", "_killed", "_event", "metadata", "_callbacks")

    def __init__(self, request_id: str | None = None, metadata: dict | None = None):
        self.id = request_id or uuid.uuid4().hex
        self._stopped = False
        self._killed = False
        self._event: asyncio.Event | None = None
        self.metadata = metadata or {}
        self._callbacks = []

    def stop_generating(self) -> None:
        """Graceful: the producer should finish the current item and stop."""
        if not self._stopped:
            self._stopped = True
            self._fire()

    def kill(self) -> None:
        """Hard: abandon the stream immediately."""
        self._killed = True
        self.stop_generating()

    def is_stopped(self) -> bool:
        return self._stopped

    def is_killed(self) -> bool:
        return self._killed

    def on_stop(self, cb) -> None:
        self._callbacks.append(cb)
        if self._stopped:
            cb()

    def _fire(self) -> None:
        if self._event is not None:
            self._event.set()
        for cb in self._callbacks:
            try:
                cb()
            except Exception:
                pass

    async def stopped(self) -> None:
        if self._stopped:
            return
        if self._event is None:
            self._event = asyncio.Event()
        await self._event.wait()

    def child(self) -> "Context":
        c = Context(self.id, dict(self.metadata))
        self.on_stop(c.stop_generating)
        return c
