"""Planner state file ~/.dynamo/state/{namespace}.json (reference
docs/planner.md:91-128): which components run, on which GPUs, under which
leases -- written by `serve` (supervisor) and the workers, read by the
planner's LocalConnector."""
from __future__ import annotations

import fcntl
import json
import os
from contextlib import contextmanager


def state_dir() -> str:
    d = os.environ.get("DYN_STATE_DIR", os.path.expanduser("~/.dynamo/state"))
    os.makedirs(d, exist_ok=True)
    return d


def state_path(namespace: str) -> str:
    return os.path.join(state_dir(), f"{namespace}.json")


@contextmanager
def locked_state(namespace: str):
    p = state_path(namespace)
    with open(p + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            st = json.load(open(p)) if os.path.exists(p) else {"components": {}, "gpus": {}}
        except json.JSONDecodeError:
            st = {"components": {}, "gpus": {}}
        yield st
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f, indent=1)
        os.replace(tmp, p)
        fcntl.flock(lk, fcntl.LOCK_UN)


def read_state(namespace: str) -> dict:
    p = state_path(namespace)
    if not os.path.exists(p):
        return {"components": {}, "gpus": {}}
    with open(p) as f:
        return json.load(f)


def record_worker(namespace: str, service: str, pid: int, lease_id: int) -> None:
    with locked_state(namespace) as st:
        comp = st["components"].setdefault(service, {"workers": {}})
        w = comp["workers"].setdefault(str(pid), {})
        w["lease"] = lease_id
        w["pid"] = pid
