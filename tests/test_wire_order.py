"""CPU checks of the wire-order protocol (disagg/agent.py): one ordered
channel, one FIFO per decode engine, no overtaking."""
import collections

from dynamo_exp_amd.disagg.agent import KVTransferAgent, WireOrder, decode_leader_hook


def test_wire_order_never_overtakes():
    w = WireOrder()
    for i in range(5):
        w.push({"i": i, "n": 2 if i == 2 else 1})
    budget = [3]

    def reserve(m):
        if m["n"] > budget[0]:
            return False
        budget[0] -= m["n"]
        return True

    assert [m["i"] for m in w.pop_ready(reserve)] == [0, 1]  # 2 needs 2, only 1 left: it and all after wait
    assert w.deferred == 1 and len(w) == 3
    budget[0] = 10
    assert [m["i"] for m in w.pop_ready(reserve)] == [2, 3, 4]


class _Pool:
    def __init__(self, ok=True):
        self.ok = ok

    def reserve(self, *n):
        return self.ok


class _DP:
    block_size = 16
    recvs: dict = {}

    def recv_bytes(self, nblocks, tp):
        return nblocks

    def send_bytes(self, nblocks, tp):
        return nblocks

    def recvs_landed(self):
        return []


class _Sched:
    remote: dict = {}


class _Eng:
    scheduler = _Sched()


def _agent(engine_id="d0"):
    a = KVTransferAgent.__new__(KVTransferAgent)
    a.engine_id, a.rank, a.tp, a.ns = engine_id, 0, 1, "ns"
    a.inbox = collections.deque()
    a.cancelled = collections.OrderedDict()
    a.cancel_seq = 0
    a.dp, a.engine = _DP(), _Eng()
    a.stats = dict(deferred=0)
    a.record_spans, a.spans = False, {}
    a.published = []
    a._publish_wire = lambda m: a.published.append(m)
    a.dp.pool = _Pool()
    return a


class _Rep:
    def __init__(self):
        self.events = []

    def submit(self, name, payload):
        self.events.append((name, payload.get("rid") if isinstance(payload, dict) and "rid" in payload
                            else [x["rid"] for x in payload["reqs"]] if isinstance(payload, dict) else payload))


def test_decode_hook_posts_in_arrival_order_across_kinds_and_sources():
    """Round 5 posted every source's starts before any read; the wire order
    keeps the control plane's order: read(p0) < start(p1) < start(p0)."""
    a = _agent()
    for m in ({"t": "read", "dst": "d0", "rid": "R", "src": "p0", "src_tp": 1, "first": 0, "last": 2},
              {"t": "start", "src": "p1", "src_tp": 1, "by_dst": {"d0": [{"rid": "A", "nblocks": 3}],
                                                                  "d1": [{"rid": "X", "nblocks": 1}]}},
              {"t": "start", "src": "p0", "src_tp": 1, "by_dst": {"d1": [{"rid": "Y", "nblocks": 1}]}},
              {"t": "start", "src": "p0", "src_tp": 1, "by_dst": {"d0": [{"rid": "B", "nblocks": 1}]}},
              {"t": "cancel", "rid": "Z"}):
        a._on_wire(m)
    assert [m["t"] for m in a.inbox] == ["read", "start", "start"]  # d1's entries are not ours
    assert a.is_cancelled("Z") and a.cancel_seq == 1
    rep = _Rep()
    hook = decode_leader_hook(rep, a, start_timeout=0)
    hook()
    assert rep.events == [("kv_read", "R"), ("kv_recv", ["A"]), ("kv_recv", ["B"])]
    # backpressure at the head holds everything behind it
    a2, rep2 = _agent(), _Rep()
    a2.dp.pool.ok = False
    a2._on_wire({"t": "start", "src": "p0", "src_tp": 1, "by_dst": {"d0": [{"rid": "A", "nblocks": 3}]}})
    a2._on_wire({"t": "read", "dst": "d0", "rid": "R", "src": "p0", "src_tp": 1, "first": 0, "last": 1})
    h2 = decode_leader_hook(rep2, a2, start_timeout=0)
    h2()
    assert rep2.events == [] and h2.pending() == 2
    a2.dp.pool.ok = True
    h2()
    assert rep2.events == [("kv_recv", ["A"]), ("kv_read", "R")]


def test_prefill_announces_one_wire_message_per_forward():
    """Every destination's entries of one forward in ONE message: one
    position in the total order for all the sends that forward enqueues."""
    from types import SimpleNamespace

    a = _agent("p0")
    a.reservations = {}

    class _DPS:
        block_size = 16
        one_sided = False

        def begin_send(self, rid, blocks, dst, dst_tp, dst_block_ids=None):
            return {"rid": rid, "nblocks": len(blocks)}

    a.dp = _DPS()
    a.tp_of = lambda e: 1
    reqs = [SimpleNamespace(request_id=f"r{i}", remote_decode=True, prompt=list(range(40)),
                            block_ids=[1, 2, 3], remote_meta={"dst": d, "dst_tp": 1, "skip": 0})
            for i, d in enumerate(["d0", "d1", "d0"])]
    batch = SimpleNamespace(requests=reqs, n_prefill=3, sample=[True, True, True])
    a.on_batch(batch)
    assert len(a.published) == 1
    m = a.published[0]
    assert m["t"] == "start" and m["src"] == "p0"
    assert {k: [x["rid"] for x in v] for k, v in m["by_dst"].items()} == {"d0": ["r0", "r2"], "d1": ["r1"]}
