"""JSONL event recorder with rotation and limits, KV-event recorder and
offline replay into an indexer (reference lib/llm/src/recorder.rs:38,
kv_router/recorder.rs, python `replay_events` lib/bindings/python/rust/llm/kv.rs:489).

Each line is `{"timestamp": <ms since recorder start>, "event": <obj>}`.
`max_lines_per_file` rotates to `path`, `path.1`, `path.2`, ...; recording
stops after `max_count` events or `max_time` seconds.
"""
from __future__ import annotations

import asyncio
import glob
import json
import os
import re
import time
from typing import Any, Iterator

from .kv_router import KV_EVENT_SUBJECT


class Recorder:
    def __init__(self, path: str, max_lines_per_file: int | None = None, max_count: int | None = None,
                 max_time: float | None = None):
        self.base = path
        self.max_lines = max_lines_per_file
        self.max_count = max_count
        self.max_time = max_time
        self.t0 = time.monotonic()
        self.count = 0
        self._lines_in_file = 0
        self._file_idx = 0
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._f = open(path, "w")

    @property
    def done(self) -> bool:
        return (self.max_count is not None and self.count >= self.max_count) or \
            (self.max_time is not None and time.monotonic() - self.t0 >= self.max_time)

    def elapsed_ms(self) -> float:
        return (time.monotonic() - self.t0) * 1000.0

    def record(self, event: Any) -> bool:
        if self._f is None or self.done:
            return False
        if self.max_lines and self._lines_in_file >= self.max_lines:
            self._f.close()
            self._file_idx += 1
            self._f = open(f"{self.base}.{self._file_idx}", "w")
            self._lines_in_file = 0
        self._f.write(json.dumps({"timestamp": round(self.elapsed_ms(), 3), "event": event}) + "\n")
        self._f.flush()
        self.count += 1
        self._lines_in_file += 1
        return True

    def files(self) -> list[str]:
        return [self.base] + [f"{self.base}.{i}" for i in range(1, self._file_idx + 1)]

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


def read_events(path: str) -> Iterator[tuple[float, Any]]:
    """Yield (timestamp_ms, event) from `path` and its rotations in order."""
    rot = sorted(glob.glob(glob.escape(path) + ".*"), key=lambda p: int(re.sub(r".*\.", "", p) or 0))
    for p in [path] + [r for r in rot if re.fullmatch(r"\d+", r.rsplit(".", 1)[1])]:
        with open(p) as f:
            for line in f:
                if line.strip():
                    d = json.loads(line)
                    yield d["timestamp"], d["event"]


class KvRecorder:
    """Records a component's `kv_events` stream."""

    def __init__(self, component, path: str, **limits):
        self.component = component
        self.rec = Recorder(path, **limits)
        self._task = None

    async def start(self) -> "KvRecorder":
        sub = await self.component.subscribe(KV_EVENT_SUBJECT)

        async def loop():
            async for ev in sub:
                if not self.rec.record(ev):
                    break

        self._task = asyncio.create_task(loop())
        return self

    @property
    def event_count(self) -> int:
        return self.rec.count

    def shutdown(self) -> None:
        if self._task:
            self._task.cancel()
        self.rec.close()


async def replay_events(path: str, indexer, timed: bool = False, speedup: float = 1.0) -> int:
    """Apply recorded router events to a KvIndexer (optionally honoring the
    recorded inter-arrival times).  Returns the number of events applied."""
    n = 0
    last = None
    for ts, ev in read_events(path):
        if timed and last is not None and ts > last:
            await asyncio.sleep((ts - last) / 1000.0 / speedup)
        last = ts
        indexer.apply(ev)
        n += 1
    return n
