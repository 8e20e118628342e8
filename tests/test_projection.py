"""tools/disagg_projection.py: the disagg-vs-agg model on toy inputs, the P->D transfer charge, and every
committed projection table (profiles/r5_disagg_projection*.json: transfer not charged; r6_*: charged)
reproduced from the measured inputs committed next to it."""
import json
import os

import pytest

from tools import disagg_projection as dp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def test_frontier_interpolates_between_pareto_points():
    pts = [(10.0, 100.0), (20.0, 80.0), (30.0, 50.0), (25.0, 40.0)]  # (25, 40) is dominated by (30, 50)
    assert dp.frontier(pts, 20.0) == 80.0
    assert dp.frontier(pts, 25.0) == pytest.approx(65.0)
    assert dp.frontier(pts, 5.0) == 100.0  # below every point: the fastest-per-GPU point
    assert dp.frontier(pts, 31.0) is None  # nothing reaches it


def test_project_decode_bound_and_prefill_bound_points():
    agg = [{"concurrency": 8, "tok_s_gpu": 100.0, "tok_s_user": 12.5}]
    # all prompts remote: the decode GPU's 150 tok/s at OSL 150 needs 1 prompt/s; 300 needs 2
    decode = {1.0: [{"concurrency": 4, "tok_s_gpu": 150.0, "tok_s_user": 37.5},
                    {"concurrency": 8, "tok_s_gpu": 300.0, "tok_s_user": 37.5}]}
    res = dp.project(agg, decode, prompts_s=1.5, osl=150)
    d = res["disagg"]
    assert d[0]["bound"] == "decode" and d[0]["tok_s_gpu"] == 75.0  # a pair of GPUs
    # the prefill GPU caps the second point: demand 2 > 1.5 -> settles halfway between the two
    assert d[1]["bound"] == "prefill" and d[1]["decode_tok_s"] == pytest.approx(225.0)
    assert d[1]["decode_concurrency"] == pytest.approx(6.0)


def test_transfer_charge():
    """each remote prompt costs the prefill GPU its wire
    time over one xGMI link plus the pack overhead, the decode GPU its unpack."""
    ch = dp.charged_rates(prompts_s=30.0, isl=3000, kv_bytes_per_token=131072, link_GBps=76.5, pack_overhead=0.007,
                          unpack_ms=0.1)
    wire = 3000 * 131072 / 76.5e9
    assert ch["wire_ms"] == pytest.approx(wire * 1e3, abs=1e-3)
    assert ch["prefill_prompts_s_charged"] == pytest.approx(1.0 / (1.007 / 30.0 + wire))
    assert dp.charged_rates(30.0, 3000, 131072, 0.0, 0.0, 0.0)["prefill_prompts_s_charged"] == pytest.approx(30.0)
    # the decode GPU's unpack scales its rate by 1 / (1 + remote prompts/s x unpack)
    decode = {1.0: [{"concurrency": 8, "tok_s_gpu": 1500.0, "tok_s_user": 50.0}]}
    res = dp.project([], decode, prompts_s=100.0, osl=150, unpack_ms=10.0)
    assert res["disagg"][0]["decode_tok_s"] == pytest.approx(1500.0 / 1.1)


def _key(r):
    return r.get("disagg_tok_s_gpu_projected", r.get("disagg_tok_s_gpu"))


@pytest.mark.parametrize("out,inputs,kv,charged", [
    ("r5_disagg_projection.json", "r5_proj", 131072, False),
    ("r5_disagg_projection_70b.json", "r5_proj70b", 327680, False),
    ("r5_disagg_projection_70b_fp8.json", "r5_proj70b_fp8", 163840, False),
    ("r6_disagg_projection.json", "r5_proj", 131072, True),
    ("r6_disagg_projection_70b.json", "r5_proj70b", 327680, True),
    ("r6_disagg_projection_70b_fp8.json", "r5_proj70b_fp8", 163840, True),
])
def test_committed_projection_tables_reproduce(out, inputs, kv, charged, capsys):
    want = json.load(open(os.path.join(PROF, out)))
    prompts_s = json.load(open(os.path.join(PROF, f"{inputs}_prefill_role.json")))["prompts_s"]
    assert prompts_s == want["prefill_prompts_s"]
    targets = ",".join(str(r["tok_s_user"]) for r in want["table"])
    decode = [os.path.join(PROF, f"{inputs}_q{q}.json") for q in ("1.0", "0.75", "0.5")]
    extra = ["--kv-bytes-per-token", str(kv)] if charged else ["--link-GBps", "0", "--pack-overhead", "0",
                                                              "--unpack-ms", "0"]
    got = dp.main(["--agg", os.path.join(PROF, f"{inputs}_agg.json"), "--decode", *decode,
                   "--prefill-prompts-s", str(prompts_s), "--osl", str(want["osl"]), "--targets", targets] + extra)
    capsys.readouterr()
    assert [(r["tok_s_user"], r["agg_tok_s_gpu"], _key(r), r["ratio"]) for r in got["table"]] == \
        [(r["tok_s_user"], r["agg_tok_s_gpu"], _key(r), r["ratio"]) for r in want["table"]]
    if charged:
        assert got["transfer_charge"]["wire_ms"] > 0 and "projection" in got["kind"]
