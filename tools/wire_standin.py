#!/usr/bin/env python3
"""Two-process WRITE + READ cross-traffic through the real KV data plane over
an RCCL stand-in wire, on ONE GPU (second half).

RCCL cannot run two ranks on one device, so `FlagLinks` gives the data plane
(disagg/transfer.py `KVDataPlane`) a wire with RCCL's point-to-point
semantics: each (src, dst, direction) channel is a stream of its own (like a
per-pair communicator's stream) whose send / recv kernels
(csrc/kernels/wire_standin.hip) each hold their hardware queue until the
peer's matching kernel runs -- rendezvous, in order per channel.  Channel
state and payload live in uncached device memory shared over IPC.  A spin
that waits longer than --timeout-ms sets the channel's error word: a deadlock
becomes exit status 3, never a hung GPU.

The scenario is the verdict's: a prefill engine posts a prefix READ receive
and then, in its next forward, the layer-streamed WRITE sends of another
request; messages reach the decode engine through an ordered channel (a
TCPStore log standing in for the control plane's wire subject).  With
GPU_MAX_HW_QUEUES=1 every stream of a process shares one queue per priority,
the worst case of queue sharing.

  --order wire    the decode side posts in arrival order (agent.WireOrder,
                  the serving code path) -> must complete, bytes verified;
  --order legacy  round 5's order (every start before any read) -> the
                  cycle; the spins time out (the test's negative control).

Run by tests/test_wire_hazards_gpu.py; by hand:
  python tools/wire_standin.py --order wire [--rounds 6]
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

L, NB, H, BS, D = 4, 128, 8, 16, 128  # a small paged KV cache [L, 2, NB, H, BS, D] bf16
WIRE_BYTES = 4 << 20
NBLK = 6  # blocks per request


class _Work:
    __slots__ = ("ev",)

    def __init__(self, ev):
        self.ev = ev

    def is_completed(self) -> bool:
        return self.ev.query()

    def wait(self) -> None:
        import torch

        torch.cuda.current_stream().wait_event(self.ev)


class FlagLinks:
    """`send` / `recv` over stand-in channels (the WorldLinks signature).
    chans[(src_engine, src_rank, dst_engine, dst_rank, rev)] = (state, wire,
    err) device pointers; every channel gets its own normal-priority stream."""

    def __init__(self, me: tuple, chans: dict, timeout_ms: int):
        import torch

        from dynamo_exp_amd import _native

        self.me, self.chans, self.timeout_ms = me, chans, timeout_ms
        self.k = _native.kernels()
        self.streams = {c: torch.cuda.Stream() for c in chans}  # normal priority, like ProcessGroupNCCL's
        self.seq = {c: 0 for c in chans}

    def _xfer(self, chan, t, send: int):
        import torch

        state, wire, err = self.chans[chan]
        nbytes = t.numel() * t.element_size()
        assert nbytes <= WIRE_BYTES and nbytes % 16 == 0, nbytes
        s = self.streams[chan]
        s.wait_stream(torch.cuda.current_stream())  # the payload is ready (a communicator stream does the same)
        k = self.seq[chan]
        self.seq[chan] = k + 1
        self.k.wire_xfer(send, state, wire, t.data_ptr(), nbytes, k, self.timeout_ms, err, s.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(s)
        return _Work(ev)

    def send(self, engine: str, rank: int, t, rev: bool = False):
        return self._xfer((self.me[0], self.me[1], engine, rank, rev), t, 1)

    def recv(self, engine: str, rank: int, t, rev: bool = False):
        return self._xfer((engine, rank, self.me[0], self.me[1], rev), t, 0)


def _read_i32(ptr: int) -> int:
    from dynamo_exp_amd import _native

    return _native.kernels().device_read_i32(ptr)


def _pattern(tag: int, device):
    """The KV cache content of a role (both processes can rebuild it)."""
    import torch

    g = torch.Generator().manual_seed(1000 + tag)
    return torch.randn(L, 2, NB, H, BS, D, generator=g).to(torch.bfloat16).to(device)


def _store(port: int, master: bool):
    import torch.distributed as dist

    return dist.TCPStore("127.0.0.1", port, 2, master, timeout=datetime.timedelta(seconds=60))


def _chan_keys():
    fwd = ("p0", 0, "d0", 0, False)  # WRITE: prefill -> decode
    rev = ("d0", 0, "p0", 0, True)  # READ: decode -> prefill (reverse direction)
    return [fwd, rev]


def role_decode(a) -> dict:
    import torch

    from dynamo_exp_amd import _native
    from dynamo_exp_amd.disagg.agent import WireOrder
    from dynamo_exp_amd.disagg.transfer import KVDataPlane

    k = _native.kernels()
    st = _store(a.port, True)
    chans, handles = {}, {}
    for c in _chan_keys():
        ctl = k.wire_alloc(64)  # state word at +0, error word at +16
        wire = k.wire_alloc(WIRE_BYTES)
        chans[c] = (ctl, wire, ctl + 16)
        handles[json.dumps(c)] = [k.ipc_get_handle(ctl).hex(), k.ipc_get_handle(wire).hex()]
    st.set("handles", json.dumps(handles))
    kv = _pattern(2, "cuda")
    links = FlagLinks(("d0", 0), chans, a.timeout_ms)
    dp = KVDataPlane(kv, links, 0, 1, H, layer_group_count=2)
    wire = WireOrder()
    legacy_starts, legacy_reads = [], []
    n_msgs = 2 * a.rounds
    got = 0
    want_recv = {}
    t_end = time.time() + a.wall_s
    while time.time() < t_end:
        while got < n_msgs:
            try:
                raw = st.get(f"msg/{got}") if st.check([f"msg/{got}"]) else None
            except Exception:  # noqa: BLE001
                raw = None
            if raw is None:
                break
            m = json.loads(raw)
            got += 1
            if a.order == "wire":
                wire.push(m)
            else:
                (legacy_starts if m["t"] == "start" else legacy_reads).append(m)
        batch = wire.pop_ready(lambda m: True) if a.order == "wire" else []
        if a.order == "legacy" and legacy_starts and legacy_reads:
            # round 5's hook: every source's starts, then the reads
            batch, legacy_starts, legacy_reads = legacy_starts + legacy_reads, [], []
        for m in batch:
            if m["t"] == "start":
                blocks = m["dst_blocks"]
                want_recv[m["rid"]] = (m["src_blocks"], blocks)
                dp.post_recv_batch("p0", 1, [(m["rid"], len(blocks), blocks)])
            else:
                dp.serve_read(m["rid"], m["src_blocks"], "p0", 1)
        for rid in dp.recvs_landed():
            dp.finish_recv(rid)
        dp.poll_recvs()
        dp.poll_served()
        if got == n_msgs and not wire.q and not legacy_starts and not legacy_reads and dp.pending() == 0:
            break
        time.sleep(0.001)
    torch.cuda.synchronize()
    errs = sum(_read_i32(c[2]) for c in chans.values())
    src = _pattern(1, "cuda")
    ok = sum(bool(torch.equal(kv[:, :, d], src[:, :, s])) for s, d in want_recv.values())
    res = {"role": "decode", "pending": dp.pending(), "errors": errs, "writes_verified": ok,
           "writes": len(want_recv), "served": dp.stats["served"]}
    st.set("decode_result", json.dumps(res))
    # the channels are this process's memory: keep it mapped until the
    # prefill side's kernels have all finished and it closed its mappings
    st.wait(["prefill_done"], datetime.timedelta(seconds=a.wall_s + 60))
    return res


def role_prefill(a) -> dict:
    import torch

    from dynamo_exp_amd import _native
    from dynamo_exp_amd.disagg.transfer import KVDataPlane

    k = _native.kernels()
    st = _store(a.port, False)
    st.wait(["handles"])
    handles = json.loads(st.get("handles"))
    chans = {}
    for key, (hc, hw) in handles.items():
        c = tuple(json.loads(key))
        ctl = k.ipc_open_handle(bytes.fromhex(hc))
        wire = k.ipc_open_handle(bytes.fromhex(hw))
        chans[c] = (ctl, wire, ctl + 16)
    kv = _pattern(1, "cuda")
    links = FlagLinks(("p0", 0), chans, a.timeout_ms)
    dp = KVDataPlane(kv, links, 0, 1, H, layer_group_count=2)
    seq = 0
    reads = {}

    def publish(m):
        nonlocal seq
        st.set(f"msg/{seq}", json.dumps(m))
        seq += 1

    for r in range(a.rounds):
        # READ of a prefix the decode engine caches (its blocks < 60), landing in our blocks 64+
        rb = [(7 * r + i) % 60 for i in range(NBLK)]
        dst = [64 + NBLK * r + i for i in range(NBLK)]  # distinct per round: every pull is verified at the end
        publish({"t": "read", "rid": f"R{r}", "src_blocks": rb})
        dp.post_read(f"R{r}", dst, "d0", 1)
        reads[f"R{r}"] = (rb, dst)
        # the next forward completes another request's prompt: announce, then stream its layer groups
        wb = [(3 * r + i) % 60 for i in range(NBLK)]
        wd = [64 + NBLK * r + i for i in range(NBLK)]
        publish({"t": "start", "rid": f"W{r}", "src_blocks": wb, "dst_blocks": wd})
        dp.begin_send(f"W{r}", wb, "d0", 1)
        for layer in range(L):
            dp.on_layer(layer)
        dp.end_forward()
    t_end = time.time() + a.wall_s
    done_reads = set()
    while time.time() < t_end and (dp.pending() or len(done_reads) < len(reads)):
        for rid in dp.reads_landed():
            dp.finish_read(rid)
            done_reads.add(rid)
        dp.poll_sends()
        dp.poll_reads()
        time.sleep(0.001)
    torch.cuda.synchronize()
    errs = sum(_read_i32(c[2]) for c in chans.values())
    src = _pattern(2, "cuda")
    ok = sum(bool(torch.equal(kv[:, :, d], src[:, :, s])) for s, d in reads.values())
    res = {"role": "prefill", "pending": dp.pending(), "errors": errs, "reads_verified": ok, "reads": len(reads)}
    for ctl, wire, _ in chans.values():
        k.ipc_close_handle(ctl)
        k.ipc_close_handle(wire)
    st.wait(["decode_result"])
    res["decode"] = json.loads(st.get("decode_result"))
    res["errors"] += res["decode"]["errors"]
    st.set("prefill_done", "1")
    return res


def run_pair(order: str, rounds: int = 6, timeout_ms: int = 4000, wall_s: float = 60.0,
             hw_queues: int = 1) -> dict:
    """Start the two role processes (prefill first reads the handles the
    decode side publishes), return the prefill side's merged report."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(hw_queues), HSA_ENABLE_IPC_MODE_LEGACY="0")
    base = [sys.executable, os.path.abspath(__file__), "--order", order, "--rounds", str(rounds), "--port",
            str(port), "--timeout-ms", str(timeout_ms), "--wall-s", str(wall_s)]
    dec = subprocess.Popen(base + ["--role", "decode"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True)
    time.sleep(0.5)
    pre = subprocess.Popen(base + ["--role", "prefill"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True)
    try:
        pout, perr = pre.communicate(timeout=wall_s + 120)
        dout, derr = dec.communicate(timeout=60)
    except subprocess.TimeoutExpired:
        pre.kill()
        dec.kill()
        raise
    lines = [ln for ln in pout.splitlines() if ln.startswith("{")]
    if pre.returncode not in (0, 3) or not lines:
        raise RuntimeError(f"prefill rc {pre.returncode}: {perr[-3000:]}\ndecode rc {dec.returncode}: {derr[-3000:]}")
    res = json.loads(lines[-1])
    res["rc"] = (pre.returncode, dec.returncode)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", choices=["prefill", "decode"], default=None)
    ap.add_argument("--order", choices=["wire", "legacy"], default="wire")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--timeout-ms", type=int, default=4000)
    ap.add_argument("--wall-s", type=float, default=60.0)
    ap.add_argument("--hw-queues", type=int, default=1)
    a = ap.parse_args()
    if a.role is None:
        print(json.dumps(run_pair(a.order, a.rounds, a.timeout_ms, a.wall_s, a.hw_queues)), flush=True)
        return
    import torch

    from dynamo_exp_amd.utils import streams

    torch.cuda.set_device(0)
    streams.enter_compute("cuda:0")  # as an engine thread: compute on the high-priority stream
    if a.rounds * NBLK > NB - 64:
        raise SystemExit("too many rounds for the cache")
    res = role_decode(a) if a.role == "decode" else role_prefill(a)
    print(json.dumps(res), flush=True)
    sys.exit(3 if res["errors"] else 0)


if __name__ == "__main__":
    main()
