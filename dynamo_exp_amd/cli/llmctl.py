"""llmctl: register OpenAI models with HTTP frontends (reference
launch/llmctl/src/main.rs:115-454).

  python -m dynamo_exp_amd.cli.llmctl http add chat-models NAME ns.comp.ep
  python -m dynamo_exp_amd.cli.llmctl http add completion NAME ns/comp/ep [--router random]
  python -m dynamo_exp_amd.cli.llmctl http list [chat-models|completion]
  python -m dynamo_exp_amd.cli.llmctl http remove chat-models NAME

Entries are `models/{chat|completion}/{name}:0` ModelEntry records without a
lease (they persist until removed); frontends (`cli.http`, `ModelWatcher`)
pick them up live.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys

from ..llm.model_card import MODELS_PREFIX, ModelEntry, model_key
from ..runtime.control_plane import ControlPlaneClient, default_address

KINDS = {"chat-models": "chat", "chat": "chat", "completion": "completion", "completions": "completion",
         "completion-models": "completion"}


def parse_endpoint(s: str) -> str:
    parts = s.replace(".", "/").split("/")
    if len(parts) != 3 or not all(parts):
        raise ValueError(f"endpoint must be ns.component.endpoint, got {s!r}")
    return "/".join(parts)


async def add(cp, kind: str, name: str, endpoint: str, router: str) -> str:
    e = ModelEntry(name, parse_endpoint(endpoint), KINDS[kind], None, router)
    key = model_key(e.model_type, name)
    await cp.put(key, e.to_json())
    return key


async def list_models(cp, kind: str | None) -> list[dict]:
    out = []
    for k, v in await cp.get_prefix(MODELS_PREFIX):
        e = ModelEntry.from_json(v)
        if kind and e.model_type != KINDS[kind]:
            continue
        out.append({"name": e.name, "type": e.model_type, "endpoint": e.endpoint, "key": k,
                    "router": e.router_mode})
    return out


async def remove(cp, kind: str, name: str) -> int:
    n = 0
    for k, v in await cp.get_prefix(f"{MODELS_PREFIX}{KINDS[kind]}/{name}:"):
        n += await cp.delete(k)
    return n


async def amain(a) -> int:
    cp = await ControlPlaneClient(a.control_plane or default_address()).connect()
    try:
        if a.op == "add":
            print(await add(cp, a.kind, a.name, a.endpoint, a.router))
        elif a.op == "list":
            rows = await list_models(cp, a.kind)
            if a.json:
                print(json.dumps(rows))
            else:
                for r in rows:
                    print(f"{r['type']:<11} {r['name']:<32} {r['endpoint']}")
        elif a.op == "remove":
            n = await remove(cp, a.kind, a.name)
            if not n:
                print(f"no {a.kind} named {a.name}", file=sys.stderr)
                return 1
        return 0
    finally:
        await cp.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="llmctl")
    ap.add_argument("--control-plane", default=None)
    ap.add_argument("--public-namespace", default="public", help="accepted for compatibility")
    sub = ap.add_subparsers(dest="group", required=True)
    http = sub.add_parser("http")
    ops = http.add_subparsers(dest="op", required=True)
    p = ops.add_parser("add")
    p.add_argument("kind", choices=sorted(KINDS))
    p.add_argument("name")
    p.add_argument("endpoint")
    p.add_argument("--router", default="round_robin", choices=["round_robin", "random"])
    p = ops.add_parser("list")
    p.add_argument("kind", nargs="?", choices=sorted(KINDS))
    p.add_argument("--json", action="store_true")
    p = ops.add_parser("remove")
    p.add_argument("kind", choices=sorted(KINDS))
    p.add_argument("name")
    a = ap.parse_args(argv)
    return asyncio.run(amain(a))


if __name__ == "__main__":
    sys.exit(main())
