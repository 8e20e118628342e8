"""Runtime configuration (reference lib/runtime/src/config.rs:25-175).

Layering, lowest to highest priority:
  defaults -> /opt/dynamo/defaults/runtime.toml -> /opt/dynamo/etc/runtime.toml
  -> $DYN_RUNTIME_CONFIG (extra TOML file) -> DYN_RUNTIME_* environment
(empty environment values are ignored).  On this runtime
`num_worker_threads` sizes the native helper pools (tokenizer / hashing /
host-side copy threads) and `max_blocking_threads` the asyncio default
executor used for blocking calls.  `WorkerConfig` reads DYN_WORKER_*.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import asdict, dataclass, fields

try:
    import tomllib as _toml  # py3.11+
except ImportError:  # pragma: no cover - 3.10 image
    import tomli as _toml

DEFAULT_FILES = ("/opt/dynamo/defaults/runtime.toml", "/opt/dynamo/etc/runtime.toml")


def is_truthy(val: str | None) -> bool:
    return (val or "").strip().lower() in ("1", "true", "on", "yes")


def env_is_truthy(name: str) -> bool:
    return is_truthy(os.environ.get(name))


def _coerce(cls, raw: dict) -> dict:
    out = {}
    for f in fields(cls):
        if f.name in raw:
            out[f.name] = type(getattr(cls(), f.name))(raw[f.name])
    return out


@dataclass
class RuntimeConfig:
    num_worker_threads: int = 16
    max_blocking_threads: int = 512

    def validate(self) -> "RuntimeConfig":
        if self.num_worker_threads < 1 or self.max_blocking_threads < 1:
            raise ValueError(f"invalid runtime config {asdict(self)}: thread counts must be >= 1")
        return self

    @classmethod
    def from_settings(cls, files: tuple[str, ...] | None = None, env: dict | None = None) -> "RuntimeConfig":
        env = os.environ if env is None else env
        merged: dict = {}
        paths = list(DEFAULT_FILES if files is None else files)
        if env.get("DYN_RUNTIME_CONFIG"):
            paths.append(env["DYN_RUNTIME_CONFIG"])
        for p in paths:
            if os.path.isfile(p):
                with open(p, "rb") as f:
                    merged.update(_toml.load(f))
        for f in fields(cls):
            v = env.get(f"DYN_RUNTIME_{f.name.upper()}")
            if v:
                merged[f.name] = v
        return cls(**_coerce(cls, merged)).validate()

    @classmethod
    def single_threaded(cls) -> "RuntimeConfig":
        return cls(1, 1)

    def install(self, loop) -> None:
        """Size the loop's default executor (blocking-call threads)."""
        loop.set_default_executor(ThreadPoolExecutor(self.max_blocking_threads, thread_name_prefix="dyn-blocking"))


@dataclass
class WorkerConfig:
    graceful_shutdown_timeout: float = 30.0

    @classmethod
    def from_settings(cls, env: dict | None = None) -> "WorkerConfig":
        env = os.environ if env is None else env
        raw = {f.name: env[f"DYN_WORKER_{f.name.upper()}"] for f in fields(cls)
               if env.get(f"DYN_WORKER_{f.name.upper()}")}
        return cls(**_coerce(cls, raw))
