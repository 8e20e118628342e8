"""HIP stream placement: which streams may share a hardware queue.

A HIP stream is not a hardware queue.  ROCm maps a process's streams onto
GPU_MAX_HW_QUEUES (4) AQL queues *per priority level*; two streams on one
queue run their kernels in submission order, so a kernel that spins -- an
RCCL send/recv waiting for its peer -- holds back every later kernel of the
other stream.  Measured on an MI355X
(profiles/r6_hwq_probe.json, tools/hwq_probe.py; a 300 ms spin on each of 8
other streams, a tiny kernel on the candidate compute stream):

* legacy default stream vs 8 normal-priority streams: stuck behind one of
  them (280 ms); a torch pool stream vs 8 more pool streams: the same;
* a HIGH-priority stream vs 8 normal-priority streams: never blocked; with 3
  more high-priority streams beside it (4 in total): never blocked.

So the engine runs every stream whose progress a serving step waits on in
the high-priority pool (`ROLES`, one queue each at GPU_MAX_HW_QUEUES = 4;
TP collectives join them, `tp_group_options`), and leaves the normal-priority
pool to the KV point-to-point traffic: torch's ProcessGroupNCCL takes its
communicator streams from the normal pool unless asked otherwise, so a
spinning KV receive can only delay other KV transfers, never a decode step,
a TP all-reduce, a KV pack/unpack or a host-tier copy.  Among RCCL streams the KV data plane stays deadlock-free by ordering
(disagg/agent.py `WireOrder`), not by queue placement.

    role        priority  what
    compute     high      every engine step (prefill, decode, graph replays)
    side        high      overlapped decode attention (models/llama.py)
    kv_copy     high      P->D pack / unpack of KV staging (disagg/transfer.py)
    host_tier   high      device <-> pinned-host KV copies (engine/host_tier.py)
    rccl TP     high      TP-group collectives (ProcessGroupNCCL is_high_priority_stream)
    rccl p2p    normal    KV send / recv communicators (torch's default)

The streams are created once per (device, role) by the native binding with an
explicit priority (not from torch's round-robin pool, whose 32 streams per
priority would be handed to any other user) and wrapped as torch external
streams; they live as long as the process.
"""
from __future__ import annotations

import logging
import threading

import torch

log = logging.getLogger("dynamo_exp_amd.streams")

ROLES = ("compute", "side", "kv_copy", "host_tier")  # <= GPU_MAX_HW_QUEUES: one high-priority queue each

_lock = threading.Lock()
_streams: dict[tuple, torch.cuda.Stream] = {}
_plan_logged: set = set()


def _dev_index(device) -> int:
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def stream(role: str, device) -> torch.cuda.Stream:
    """The process's high-priority stream for `role` on `device`."""
    if role not in ROLES:
        raise ValueError(f"unknown stream role {role!r} (one of {ROLES})")
    idx = _dev_index(device)
    key = (idx, role)
    s = _streams.get(key)
    if s is not None:
        return s
    with _lock:
        s = _streams.get(key)
        if s is None:
            from .. import _native

            k = _native.kernels()
            _, hi = k.stream_priority_range()  # (least, greatest): greatest = numerically lowest = highest
            with torch.cuda.device(idx):
                h = k.stream_create(hi, 0)
            s = torch.cuda.ExternalStream(h, device=torch.device("cuda", idx))
            _streams[key] = s
    return s


def enter_compute(device) -> torch.cuda.Stream | None:
    """Make this thread's current stream the high-priority compute stream
    (idempotent, cheap).  The first switch orders the compute stream after
    what the thread's previous stream (the legacy default stream: model
    load, KV allocation) had enqueued."""
    d = torch.device(device)
    if d.type != "cuda":
        return None
    s = stream("compute", d)
    cur = torch.cuda.current_stream(d)
    if cur.cuda_stream != s.cuda_stream:
        s.wait_stream(cur)
        torch.cuda.set_stream(s)
    return s


def plan(device) -> dict:
    """The stream plan of this process on `device`: the high-priority roles
    created so far (handle, priority) and the pool RCCL uses."""
    idx = _dev_index(device)
    out = {}
    for (i, role), s in sorted(_streams.items()):
        if i == idx:
            out[role] = {"handle": hex(s.cuda_stream), "priority": "high"}
    out["rccl_tp"] = {"priority": "high", "source": "ProcessGroupNCCL is_high_priority_stream (tp_group_options)"}
    out["rccl_p2p"] = {"priority": "normal", "source": "ProcessGroupNCCL default stream pool"}
    return out


def log_plan(device, who: str = "engine") -> None:
    """Log the plan once per (device, who) -- at engine start."""
    d = torch.device(device)
    if d.type != "cuda" or (d, who) in _plan_logged:
        return
    _plan_logged.add((d, who))
    log.info("%s streams on %s: %s", who, d, plan(d))


def tp_group_options(backend: str):
    """ProcessGroupNCCL options for a TENSOR-PARALLEL group: its collective
    streams come from the high-priority pool.  A TP all-reduce is on the
    critical path of every step (the compute stream waits for it) and its
    peers run in lockstep, so it must not sit behind a spinning KV receive
    in the normal pool; the KV point-to-point communicators keep the default
    (normal) priority.  None for gloo."""
    if backend != "nccl":
        return None
    import torch.distributed as dist

    o = dist.ProcessGroupNCCL.Options()
    o.is_high_priority_stream = True
    return o
