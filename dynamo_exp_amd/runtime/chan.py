"""Single-consumer async channel for per-token streams.

asyncio.Queue does more than a token stream needs (maxsize, a getters deque
of futures, task accounting); a stream has exactly one reader, so a deque
plus at most one waiting future is enough, and costs about half as much per
item on the serving hot path (engine -> worker endpoint, request-plane
connection -> response stream)."""
from __future__ import annotations

import asyncio
from collections import deque


class Chan:
    __slots__ = ("items", "waiter")

    def __init__(self):
        self.items: deque = deque()
        self.waiter: asyncio.Future | None = None

    def put_nowait(self, item) -> None:
        self.items.append(item)
        w = self.waiter
        if w is not None:
            self.waiter = None
            if not w.done():
                w.set_result(None)

    async def get(self):
        while not self.items:
            w = self.waiter = asyncio.get_running_loop().create_future()
            try:
                await w
            finally:
                if self.waiter is w:
                    self.waiter = None
        return self.items.popleft()

    def get_nowait(self):
        if not self.items:
            raise asyncio.QueueEmpty
        return self.items.popleft()

    def qsize(self) -> int:
        return len(self.items)

    def empty(self) -> bool:
        return not self.items
