"""Logging honoring the reference's env knobs (lib/runtime/src/logging.rs:62-142):
DYN_LOG (level or `level,target=level,...` filter), DYN_LOGGING_JSONL (JSON
lines), DYN_LOG_USE_LOCAL_TZ, DYN_SDK_DISABLE_ANSI_LOGGING."""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_configured = False

_LEVELS = {"trace": 5, "debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING,
           "warning": logging.WARNING, "error": logging.ERROR}


def _truthy(v: str | None) -> bool:
    return (v or "").lower() in ("1", "true", "on", "yes")


class JsonlFormatter(logging.Formatter):
    def format(self, r: logging.LogRecord) -> str:
        ts = time.localtime(r.created) if _truthy(os.environ.get("DYN_LOG_USE_LOCAL_TZ")) else time.gmtime(r.created)
        d = {"time": time.strftime("%Y-%m-%dT%H:%M:%S", ts) + f".{int(r.msecs):03d}" +
             ("" if _truthy(os.environ.get("DYN_LOG_USE_LOCAL_TZ")) else "Z"),
             "level": r.levelname, "target": r.name, "message": r.getMessage()}
        if r.exc_info:
            d["exception"] = self.formatException(r.exc_info)
        return json.dumps(d)


def configure_logging(default: str = "info") -> None:
    global _configured
    if _configured:
        return
    _configured = True
    spec = os.environ.get("DYN_LOG", default)
    parts = [p.strip() for p in spec.split(",") if p.strip()]
    root_level = logging.INFO
    targets = {}
    for p in parts:
        if "=" in p:
            t, lv = p.split("=", 1)
            targets[t.replace("::", ".")] = _LEVELS.get(lv.lower(), logging.INFO)
        else:
            root_level = _LEVELS.get(p.lower(), logging.INFO)
    h = logging.StreamHandler(sys.stderr)
    if _truthy(os.environ.get("DYN_LOGGING_JSONL")):
        h.setFormatter(JsonlFormatter())
    else:
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(root_level)
    for t, lv in targets.items():
        logging.getLogger(t).setLevel(lv)
