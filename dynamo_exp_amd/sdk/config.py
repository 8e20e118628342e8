"""Graph configuration (reference deploy/dynamo/sdk/src/dynamo/sdk/lib/config.py).

YAML layout:
    Common:                 # shared keys, opted into per service via `common-configs`
      model: llama3-8b
    Frontend:
      port: 8000
      ServiceArgs: {workers: 1, resources: {gpu: 0}}
    VllmWorker:
      common-configs: [model]
      ServiceArgs: {workers: 2, resources: {gpu: 1}}

The resolved config travels to every worker process as the
DYNAMO_SERVICE_CONFIG env var (JSON); `as_args(service)` renders a service's
keys (+ subscribed Common keys it does not override) as `--key value` argv.
"""
from __future__ import annotations

import json
import os
from typing import Any

import yaml

ENV = "DYNAMO_SERVICE_CONFIG"
COMMON = "Common"
COMMON_KEY = "common-configs"


class ServiceConfig(dict):
    _instance: "ServiceConfig | None" = None

    @classmethod
    def get_instance(cls) -> "ServiceConfig":
        if cls._instance is None:
            raw = os.environ.get(ENV)
            cls._instance = cls(json.loads(raw) if raw else {})
        return cls._instance

    @classmethod
    def reset(cls) -> None:
        cls._instance = None

    def require(self, service: str, key: str):
        if service not in self or key not in self[service]:
            raise ValueError(f"{service}.{key} must be specified in configuration")
        return self[service][key]

    def as_args(self, service: str, prefix: str = "") -> list[str]:
        if service not in self:
            return []
        args: list[str] = []

        def add(key: str, value: Any):
            if prefix and not key.startswith(prefix):
                return
            if key.endswith(COMMON_KEY):
                return
            k = key[len(prefix):] if prefix else key
            if isinstance(value, bool):
                if value:
                    args.append(f"--{k}")
            elif isinstance(value, (dict, list)):
                args.extend([f"--{k}", json.dumps(value)])
            else:
                args.extend([f"--{k}", str(value)])

        svc = {k: v for k, v in self[service].items() if k != "ServiceArgs"}
        common = self.get(COMMON)
        keys = svc.get(COMMON_KEY)
        if common is not None and keys is not None:
            for k in keys:
                if k in common and k not in svc:
                    add(k, common[k])
        for k, v in svc.items():
            add(k, v)
        return args

    def service_args(self, service: str) -> dict:
        return dict((self.get(service) or {}).get("ServiceArgs") or {})


def _coerce(v: str):
    try:
        return json.loads(v)
    except (json.JSONDecodeError, ValueError):
        return v


def resolve(config_file: str | None, overrides: list[str] | None = None) -> dict:
    """YAML + `--Service.key=value` overrides (reference cli/serve.py:99-127)."""
    cfg: dict = {}
    if config_file:
        with open(config_file) as f:
            cfg = yaml.safe_load(f) or {}
    for o in overrides or []:
        o = o.lstrip("-")
        if "=" not in o:
            raise ValueError(f"override {o!r} must be --Service.key=value")
        path, val = o.split("=", 1)
        svc, _, key = path.partition(".")
        node = cfg.setdefault(svc, {})
        parts = key.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = _coerce(val)
    return cfg
