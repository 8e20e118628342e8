#!/usr/bin/env python3
"""How large an allocation can hipIpcOpenMemHandle import?  (round 6, the
one-sided KV transport)

The two-process one-sided bench on one GPU sat minutes inside the prefill
rank's hipIpcOpenMemHandle of the decode rank's KV cache.  A first probe
(round 6, profiles/r6_ipc_probe.json) showed the open of a 64 MiB torch
allocation return in 0.2 ms whether the exporting process sleeps or polls the
device, and the open of a 2.5 GiB allocation not return at all.  This probe
finds the size where imports stop working: ONE exporter / importer pair, the
exporter allocates buffers of ascending sizes and exports each; the importer
opens them in that order, each with --limit seconds (the binding releases the
GIL, so a stuck open is seen from a second thread), and stops at the first
that does not return.  Each mapping is checked by reading its first and last
word (device_read_i32).

    python tools/ipc_probe.py [--limit 10] [--out gpurun_out/ipc_probe_sizes.json]
    python tools/ipc_probe.py --vmm-gib 6 [--out ...]   # disagg/kv_share.py instead

--vmm-gib N checks the replacement (disagg/kv_share.py): the exporter
allocates N GiB as a SharedKVBuffer (512 MiB VMM chunks), fills the first and
last words through its torch view and serves the chunk fds on a Unix socket;
the importer maps them (RemoteMapping), reads both words, writes two words of
its own through a torch view of the mapping, and the exporter reads those.
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

MIB = 1 << 20
SIZES = [256 * MIB, 1024 * MIB, 2047 * MIB, 2049 * MIB, 4095 * MIB, 4097 * MIB, 8192 * MIB]


def _say(who, msg):
    print(f"[{time.strftime('%H:%M:%S')} {who}] {msg}", file=sys.stderr, flush=True)


def _word(b: int) -> int:
    v = b * 0x01010101
    return v - (1 << 32) if v >= 1 << 31 else v


def _exporter(q_out, q_in, sizes):
    import torch

    from dynamo_exp_amd import _native

    k = _native.kernels()
    keep = []
    for i, n in enumerate(sizes):
        buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        buf[:4096].fill_(i + 1)
        buf[-4096:].fill_(i + 101)
        keep.append(buf)
        torch.cuda.synchronize()
        base, off = k.alloc_base_offset(buf.data_ptr())
        q_out.put((n, k.ipc_get_handle(base), off))
    _say("exporter", f"exported {len(sizes)} buffers")
    q_in.get(timeout=900)  # "done"
    _say("exporter", "done")
    os._exit(0)


def _importer(q_in, q_out, res_q, limit, nsizes):
    import torch

    from dynamo_exp_amd import _native

    k = _native.kernels()
    torch.zeros(1, device="cuda:0")
    _say("importer", "ready")
    rows = []
    for i in range(nsizes):
        n, handle, off = q_in.get(timeout=600)
        out = {"bytes": n, "mib": n // MIB}

        def do_open(out=out, handle=handle):
            t0 = time.perf_counter()
            try:
                out["ptr"] = k.ipc_open_handle(handle)
                out["open_s"] = round(time.perf_counter() - t0, 4)
            except Exception as e:  # noqa: BLE001
                out["error"] = repr(e)

        th = threading.Thread(target=do_open, daemon=True)
        th.start()
        th.join(limit)
        if th.is_alive():
            out["hung_after_s"] = limit
            rows.append(out)
            _say("importer", f"{n // MIB} MiB: open did not return in {limit}s -- stopping")
            break
        if "ptr" in out:
            p = out.pop("ptr") + off
            out["bytes_ok"] = (k.device_read_i32(p) == _word(i + 1)
                               and k.device_read_i32(p + n - 4) == _word(i + 101))
        rows.append(out)
        _say("importer", f"{out}")
    res_q.put(rows)
    q_out.put("done")
    for q in (q_out, res_q):
        q.close()
        q.join_thread()
    os._exit(0)


def _vmm_exporter(q_out, q_in, gib):
    import torch

    from dynamo_exp_amd.disagg.kv_share import SharedKVBuffer

    n = gib << 30
    buf = SharedKVBuffer(n, torch.device("cuda:0"))
    t = buf.tensor((n // 4,), torch.int32)
    t[0] = 1234567
    t[-1] = 7654321
    torch.cuda.synchronize()
    q_out.put((buf.serve("probe"), n))
    _say("exporter", f"serving {buf.total >> 20} MiB in {buf.total // buf.chunk} chunks")
    q_in.get(timeout=300)  # the importer wrote its words
    got = [int(t[1].item()), int(t[-2].item())]
    q_out.put(got)
    _say("exporter", f"read back {got}")
    q_in.get(timeout=60)
    buf.close()
    os._exit(0)


def _vmm_importer(q_in, q_out, res_q, limit):
    import torch

    from dynamo_exp_amd import _native
    from dynamo_exp_amd.disagg.kv_share import RemoteMapping, _CAI

    k = _native.kernels()
    torch.zeros(1, device="cuda:0")
    from dynamo_exp_amd.disagg import kv_share

    addr, n = q_in.get(timeout=600)
    out = {"vmm_bytes": n}
    t0 = time.perf_counter()
    fds, chunk, total = kv_share._recv_fds(addr)
    _say("importer", f"received {len(fds)} fds, chunk {chunk >> 20} MiB")
    m = RemoteMapping.__new__(RemoteMapping)
    m._k = k
    m.ptr, m.total, m._handles = k.vmm_import(fds, chunk, 0)
    m.chunk = chunk
    out["map_s"] = round(time.perf_counter() - t0, 4)
    _say("importer", f"mapped in {out['map_s']} s")
    out["first_last_ok"] = (k.device_read_i32(m.ptr) == 1234567 and k.device_read_i32(m.ptr + n - 4) == 7654321)
    _say("importer", f"first / last words ok: {out['first_last_ok']}")
    v = torch.as_tensor(_CAI(m.ptr, n, m), device="cuda:0").view(torch.int32)
    v[1] = 42
    v[-2] = 43
    torch.cuda.synchronize()
    q_out.put("written")
    got = q_in.get(timeout=120)
    out["peer_sees_writes"] = got == [42, 43]
    _say("importer", f"{out}")
    m.close()
    q_out.put("done")
    res_q.put(out)
    for q in (q_out, res_q):
        q.close()
        q.join_thread()
    os._exit(0)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--limit", type=float, default=10.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--vmm-gib", type=int, default=0)
    a = ap.parse_args(argv)
    ctx = mp.get_context("spawn")
    a2b, b2a, res = ctx.Queue(), ctx.Queue(), ctx.Queue()
    if a.vmm_gib:
        pe = ctx.Process(target=_vmm_exporter, args=(a2b, b2a, a.vmm_gib))
        pi = ctx.Process(target=_vmm_importer, args=(a2b, b2a, res, a.limit))
    else:
        pe = ctx.Process(target=_exporter, args=(a2b, b2a, SIZES))
        pi = ctx.Process(target=_importer, args=(a2b, b2a, res, a.limit, len(SIZES)))
    pe.start()
    pi.start()
    rows, t0 = None, time.time()
    while rows is None and time.time() - t0 < 600:
        try:
            rows = res.get(timeout=20)
        except Exception:  # noqa: BLE001 -- queue.Empty: heartbeat
            _say("parent", f"waiting ({time.time() - t0:.0f} s)")
            if not pi.is_alive() or not pe.is_alive():
                rows = [{"error": f"a probe process died: importer exit {pi.exitcode}, exporter exit {pe.exitcode}"}]
    for p in (pi, pe):
        p.join(20)
        if p.is_alive():
            p.kill()
    print(json.dumps(rows), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"vmm" if a.vmm_gib else "sizes": rows}, f, indent=1)


if __name__ == "__main__":
    main()
