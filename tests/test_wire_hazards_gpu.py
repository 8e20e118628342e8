"""The P->D RCCL data plane under hardware-queue sharing.

* A decode rank's exact stream set with a spinning stand-in of an RCCL
  receive on every point-to-point stream: the captured decode graph replays
  at its idle speed (utils/streams.py puts every stream a step waits on in the
  high-priority queue pool; measured mapping: profiles/r6_hwq_probe.json).
* Two processes, WRITE + READ cross traffic through the real KVDataPlane over
  a rendezvous stand-in wire with RCCL's semantics, GPU_MAX_HW_QUEUES=1 (all
  of a process's streams on one queue per priority): the serving order
  (agent.WireOrder) completes with every byte verified; round 5's order
  (starts before reads) deadlocks -- seen as the stand-in's timeouts, which
  is the negative control that shows the test can see the hazard.
* The reference's benchmark layout's prefill worker (TP1, fp8, 70B layer
  shapes) starts with the memory fraction it is given.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _probe(scenario: str) -> dict:
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "hwq_probe.py"), "--scenario", scenario],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps(out))
    return out


@pytest.mark.gpu
def test_decode_graph_replays_at_idle_speed_while_p2p_streams_spin():
    r = _probe("graph")
    assert r["gpu_max_hw_queues"] == "4" and r["n_p2p_spinning"] == 9
    assert r["measured_while_spinning"], r
    assert r["ratio"] <= 1.05, r  # within 5 % of the idle replay time
    assert r["stream_plan"]["compute"]["priority"] == "high"


@pytest.mark.gpu
def test_wire_order_cross_traffic_completes_and_legacy_order_deadlocks():
    from tools.wire_standin import run_pair

    ok = run_pair("wire", rounds=6, timeout_ms=4000, wall_s=60, hw_queues=1)
    print(json.dumps(ok))
    assert ok["errors"] == 0 and ok["pending"] == 0, ok
    assert ok["reads_verified"] == ok["reads"] == 6, ok
    assert ok["decode"]["writes_verified"] == ok["decode"]["writes"] == 6, ok
    bad = run_pair("legacy", rounds=2, timeout_ms=2000, wall_s=40, hw_queues=1)
    print(json.dumps(bad))
    assert bad["errors"] > 0, bad  # the spins timed out: the order of round 5 is a deadlock here


@pytest.mark.gpu
def test_tp1_fp8_prefill_worker_of_70b_shapes_uses_its_memory_flag(cuda):
    import torch

    from dynamo_exp_amd.llm.workers import _engine, parse_worker_args
    from dynamo_exp_amd.engine.request import SamplingParams

    a = parse_worker_args(["--model", "llama3-70b@8", "--quantization", "fp8", "--kv-cache-dtype", "fp8",
                           "--max-model-len", "3500", "--gpu-memory-utilization", "0.9", "--block-size", "64"])
    rep = _engine(a, prefill_only=True)
    eng = rep.engine
    try:
        assert eng.cfg.gpu_memory_utilization == 0.9 and eng.cfg.max_num_seqs == 32
        free, total = torch.cuda.mem_get_info(cuda)
        kv = eng.runner.kv_bytes
        # weights of 8 layers + embeddings are ~11 GB: a 0.5 budget would give the KV < 0.5 of the device
        assert kv > 0.6 * total, (kv / 2**30, total / 2**30)
        outs = []
        eng.add_request("p", list(range(100, 3100)), SamplingParams(max_tokens=1, ignore_eos=True),
                        on_output=lambda r, t, lp, fin: outs.extend(t))
        while eng.has_unfinished():
            eng.step()
        assert len(outs) == 1
    finally:
        del rep, eng
        torch.cuda.empty_cache()
