"""tools/disagg_projection.py: the disagg-vs-agg model on toy inputs, and every committed projection table
(profiles/r5_disagg_projection*.json) reproduced from the measured inputs committed next to it."""
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


@pytest.mark.parametrize("out,inputs", [
    ("r5_disagg_projection.json", "r5_proj"),
    ("r5_disagg_projection_70b.json", "r5_proj70b"),
    ("r5_disagg_projection_70b_fp8.json", "r5_proj70b_fp8"),
])
def test_committed_projection_tables_reproduce(out, inputs, capsys):
    want = json.load(open(os.path.join(PROF, out)))
    prompts_s = json.load(open(os.path.join(PROF, f"{inputs}_prefill_role.json")))["prompts_s"]
    assert prompts_s == want["prefill_prompts_s"]
    targets = ",".join(str(r["tok_s_user"]) for r in want["table"])
    decode = [os.path.join(PROF, f"{inputs}_q{q}.json") for q in ("1.0", "0.75", "0.5")]
    got = dp.main(["--agg", os.path.join(PROF, f"{inputs}_agg.json"), "--decode", *decode,
                   "--prefill-prompts-s", str(prompts_s), "--osl", str(want["osl"]), "--targets", targets])
    capsys.readouterr()
    assert [(r["tok_s_user"], r["agg_tok_s_gpu"], r["disagg_tok_s_gpu"], r["ratio"]) for r in got["table"]] == \
        [(r["tok_s_user"], r["agg_tok_s_gpu"], r["disagg_tok_s_gpu"], r["ratio"]) for r in want["table"]]
