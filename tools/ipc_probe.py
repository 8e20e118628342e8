#!/usr/bin/env python3
"""When does hipIpcOpenMemHandle return?  (round 6, the one-sided KV transport)

The two-process one-sided bench on one GPU sat ~3 minutes inside the prefill
rank's hipIpcOpenMemHandle of the decode rank's KV cache while the decode rank
waited in a gloo barrier.  This probe runs exporter / importer process pairs
(fresh pair per case) and times the importer's open while the exporter:

  sleep     sleeps in Python (no HIP call at all)
  poll      calls torch.cuda.synchronize() every millisecond
  opening   opens a handle of the importer's buffer at the same time (the
            custom all-reduce's handshake, which is known to work)

for a small (64 MiB) and a large (2.5 GiB) torch allocation.  An open that
has not returned after --limit seconds is reported as hung and the pair is
ended with os._exit (a host-side wait; nothing is launched on the GPU).

    python tools/ipc_probe.py [--limit 20] [--out gpurun_out/ipc_probe.json]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _exporter(nbytes, mode, q_out, q_in, limit):
    import torch

    from dynamo_exp_amd import _native

    k = _native.kernels()
    buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0")
    buf[:16] = 7
    torch.cuda.synchronize()
    base, off = k.alloc_base_offset(buf.data_ptr())
    q_out.put(("handle", k.ipc_get_handle(base), off, os.getpid()))
    t0 = time.time()
    if mode == "opening":
        other = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
        ob, oo = k.alloc_base_offset(other.data_ptr())
        q_out.put(("handle2", k.ipc_get_handle(ob), oo, os.getpid()))
        msg = q_in.get(timeout=limit + 30)
        p = k.ipc_open_handle(msg[1])
        k.ipc_close_handle(p)
    while time.time() - t0 < limit + 5:
        try:
            msg = q_in.get_nowait()
            if msg == "done":
                break
        except Exception:  # noqa: BLE001 -- queue.Empty
            pass
        if mode == "poll":
            torch.cuda.synchronize()
            time.sleep(0.001)
        else:
            time.sleep(0.05)
    os._exit(0)


def _importer(q_in, q_out, mode, limit, res_q):
    import torch

    from dynamo_exp_amd import _native

    k = _native.kernels()
    torch.zeros(1, device="cuda:0")
    msg = q_in.get(timeout=120)
    if mode == "opening":
        mine = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
        mb, mo = k.alloc_base_offset(mine.data_ptr())
        q_out.put(("handle", k.ipc_get_handle(mb), mo, os.getpid()))
        q_in.get(timeout=60)  # the exporter's second handle (ignored)
    out = {}

    def do_open():
        t0 = time.perf_counter()
        try:
            p = k.ipc_open_handle(msg[1])
            out["open_s"] = round(time.perf_counter() - t0, 4)
            out["ok"] = True
            k.ipc_close_handle(p)
        except Exception as e:  # noqa: BLE001
            out["error"] = repr(e)

    th = threading.Thread(target=do_open, daemon=True)
    th.start()
    th.join(limit)
    if th.is_alive():
        out["hung_s"] = limit
    q_out.put("done")
    res_q.put(out)
    os._exit(0)


def run_case(nbytes, mode, limit):
    ctx = mp.get_context("spawn")
    a2b, b2a, res = ctx.Queue(), ctx.Queue(), ctx.Queue()
    pe = ctx.Process(target=_exporter, args=(nbytes, mode, a2b, b2a, limit))
    pi = ctx.Process(target=_importer, args=(a2b, b2a, mode, limit, res))
    pe.start()
    pi.start()
    try:
        out = res.get(timeout=limit + 180)
    except Exception as e:  # noqa: BLE001
        out = {"error": f"no result: {e!r}"}
    for p in (pi, pe):
        p.join(30)
        if p.is_alive():
            p.kill()
    return {"mode": mode, "bytes": nbytes, **out}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--limit", type=float, default=20.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--modes", default="opening,poll,sleep")
    a = ap.parse_args(argv)
    rows = []
    for mode in a.modes.split(","):
        for nbytes in (64 << 20, 2560 << 20):
            r = run_case(nbytes, mode, a.limit)
            print(json.dumps(r), flush=True)
            rows.append(r)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
