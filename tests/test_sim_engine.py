"""The MI355X timing model (engine/sim.py) in its disaggregation roles, and
the bulk two-part frame reader of the request plane."""
import asyncio

from dynamo_exp_amd.engine.request import SamplingParams
from dynamo_exp_amd.engine.sim import SimLLMEngine


def test_sim_calibration_and_metrics():
    e = SimLLMEngine.mi355x_8b("decode", host_ms=0.0)
    assert e.decode_ms == 6.5 and abs(e.decode_per_seq_ms - 0.064) < 1e-9 and e.prefill_tok_per_ms == 94.7
    assert e.num_blocks > 20000  # 0.9 of 288 GB of 64-token Llama-3-8B blocks
    for i in range(3):
        e.add_request(f"r{i}", list(range(100)), SamplingParams(max_tokens=4, ignore_eos=True))
    e.step()
    m = e.forward_pass_metrics()
    assert m["request_active_slots"] == 3 and m["kv_active_blocks"] == 3 * 2 and m["num_requests_waiting"] == 0
    while e.has_unfinished():
        e.step()
    assert e.stats["generated_tokens"] == 12


def test_sim_disaggregated_roles():
    """Decode engine parks a remote-prefill request and announces it; the
    prefill engine prefills a remote-decode request and hands it off; the
    decode engine finishes it with the prefill worker's first token."""
    d = SimLLMEngine.mi355x_8b("decode", host_ms=0.0)
    p = SimLLMEngine.mi355x_8b("prefill", host_ms=0.0)
    announced, handed = [], []
    d.scheduler.on_remote_prefill = announced.append
    p.prefill_done_hook = handed.append
    out = []
    d.add_request("x", list(range(3000)), SamplingParams(max_tokens=5, ignore_eos=True),
                  on_output=lambda r, t, lp, fin: out.extend(t), remote_prefill=True)
    d.step()
    assert [r.request_id for r in announced] == ["x"] and "x" in d.remote
    assert d.forward_pass_metrics()["kv_active_blocks"] == 3000 // 64 + 1
    p.add_request("x", list(range(3000)), SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True,
                  remote_meta={"dst": "d0"})
    p.step()
    assert len(handed) == 1 and not p.has_unfinished() and p.timing["device"] >= 3000 / 94.7 / 1000
    d.finish_remote_prefill("x", handed[0].output[0], 0.0)
    while d.has_unfinished():
        d.step()
    assert len(out) == 5 and out[0] == handed[0].output[0]


def test_iter_two_part_bulk_reader():
    from dynamo_exp_amd.runtime.wire import TwoPartError, encode_two_part, iter_two_part

    frames = [(f"h{i}".encode(), bytes([i % 251]) * (i * 37 % 3000)) for i in range(200)]
    blob = b"".join(encode_two_part(h, b) for h, b in frames)

    async def run(data, chunk):
        r = asyncio.StreamReader()
        for i in range(0, len(data), chunk):  # arbitrary fragmentation
            r.feed_data(data[i:i + chunk])
        r.feed_eof()
        got = []
        try:
            async for hb, body in iter_two_part(r, chunk=chunk):
                got.append((hb, body))
        except asyncio.IncompleteReadError:
            pass
        return got

    for chunk in (7, 1000, 1 << 18):
        assert asyncio.run(run(blob, chunk)) == frames
    bad = bytearray(blob)
    bad[30] ^= 0xFF
    try:
        asyncio.run(run(bytes(bad), 4096))
        raise AssertionError("corrupt frame accepted")
    except TwoPartError:
        pass
