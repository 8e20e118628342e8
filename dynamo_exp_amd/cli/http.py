"""Standalone OpenAI HTTP frontend (reference components/http/src/main.rs:38-103).

  python -m dynamo_exp_amd.cli.http [--host 0.0.0.0] [--port 8080] [--control-plane host:port]
                                    [--router-mode round_robin|random|kv] [--request-template t.json]

Serves every model registered on the control plane: `backend` entries from
workers (`attach`) get a local preprocessor + router pipeline, `chat` /
`completion` entries from `llmctl` forward raw OpenAI requests.
"""
from __future__ import annotations

import argparse
import asyncio

from ..llm.discovery import ModelWatcher
from ..llm.http_service import HttpService, RequestTemplate
from ..runtime import DistributedRuntime, configure_logging


async def serve(a) -> None:
    drt = await DistributedRuntime.create(a.control_plane, is_static=True)
    tmpl = RequestTemplate.load(a.request_template) if a.request_template else None
    svc = HttpService(a.host, a.port, request_template=tmpl, reuse_port=a.reuse_port)
    watcher = await ModelWatcher(drt, svc.manager, a.router_mode).start()
    try:
        await svc.run()
    finally:
        if watcher._task:
            watcher._task.cancel()
        await drt.close(1)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="http")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--control-plane", default=None)
    ap.add_argument("--router-mode", default=None, choices=[None, "round_robin", "random", "kv"])
    ap.add_argument("--request-template", default=None)
    ap.add_argument("--reuse-port", action="store_true",
                    help="SO_REUSEPORT: run several frontend processes on one port")
    a = ap.parse_args(argv)
    configure_logging()
    asyncio.run(serve(a))


if __name__ == "__main__":
    main()
