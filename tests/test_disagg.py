"""Disaggregated prefill/decode correctness on CPU.

* in-process: a prefill engine computes the prompt, its KV blocks are packed,
  "transferred" and unpacked into a decode engine's blocks (with a prefix hit
  on the decode side), and decoding produces exactly the tokens of a single
  aggregated engine;
* multi-process: the real xPyD benchmark path (torchrun, gloo p2p standing in
  for RCCL, control-plane prefill queue) runs 1P1D end to end.
"""
import os
import subprocess
import sys

import pytest
import torch

from dynamo_exp_amd.disagg.router import DisaggregatedRouter
from dynamo_exp_amd.disagg.transfer import pack_blocks, transfer_bytes, unpack_blocks
from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine(model=None, blocks=300, kv_cache_dtype="auto"):
    return LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=16, max_model_len=512,
                                  num_gpu_blocks=blocks, max_num_seqs=8, seed=5, kv_cache_dtype=kv_cache_dtype),
                     model=model)


def _run(e, rid, prompt, n, **kw):
    out = []
    e.add_request(rid, prompt, SamplingParams(max_tokens=n, ignore_eos=True),
                  on_output=lambda r, t, lp, fin: out.extend(t), **kw)
    while e.has_unfinished():
        e.step()
    return out


@pytest.mark.parametrize("kvd", ["auto", "fp8"])
def test_pack_unpack_roundtrip(kvd):
    e = _engine(kv_cache_dtype=kvd)
    kv = e.runner.kv_cache
    kv.copy_(torch.randn_like(kv.float()).to(kv.dtype))
    buf = pack_blocks(kv, [5, 9, 2])
    assert buf.numel() == transfer_bytes(kv, 3)
    kv2 = torch.zeros_like(kv)
    unpack_blocks(kv2, buf, [0, 1, 2])
    assert torch.equal(kv2[:, :, :3].view(torch.uint8), kv[:, :, [5, 9, 2]].view(torch.uint8))


@pytest.mark.parametrize("kvd", ["auto", "fp8"])
def test_remote_prefill_matches_aggregated(kvd):
    """The P->D block transfer (also with an e4m3 KV cache: raw bytes move)."""
    agg = _engine(kv_cache_dtype=kvd)
    prompt = list(range(20, 20 + 150))
    shared = prompt[:64]
    ref = _run(agg, "a", prompt, 10)

    prefill = _engine(model=agg.model, kv_cache_dtype=kvd)
    decode = _engine(model=agg.model, kv_cache_dtype=kvd)
    # warm the decode side's prefix cache with a request sharing 64 tokens
    _run(decode, "warm", shared + [7] * 10, 2)

    got = []
    decode.add_request("x", prompt, SamplingParams(max_tokens=10, ignore_eos=True),
                       on_output=lambda r, t, lp, fin: got.extend(t), remote_prefill=True)
    decode.step()  # allocates blocks, parks the request
    dreq = decode.scheduler.remote["x"]
    skip = dreq.num_computed // 16
    assert skip == 4  # 64 shared tokens hit the decode-side prefix cache
    sent = {}
    prefill.prefill_done_hook = lambda r: sent.setdefault("req", r)
    prefill.add_request("x", prompt, SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True)
    while "req" not in sent:
        prefill.step()
    preq = sent["req"]
    nblk = (len(prompt) + 15) // 16
    buf = pack_blocks(prefill.runner.kv_cache, preq.block_ids[skip:nblk])
    unpack_blocks(decode.runner.kv_cache, buf, dreq.block_ids[skip:nblk])
    prefill.finish_transfer("x")
    assert not prefill.has_unfinished()
    decode.finish_remote_prefill("x", preq.output[0], preq.logprobs[0])
    while decode.has_unfinished():
        decode.step()
    assert got == ref


def test_disagg_router_policy():
    r = DisaggregatedRouter(max_local_prefill_length=1000, max_prefill_queue_size=2)
    assert r.prefill_remote(3000, 0, 0)
    assert not r.prefill_remote(3000, 2500, 0)  # prefix hit keeps it local
    assert not r.prefill_remote(3000, 0, 2)  # queue full
    assert not r.prefill_remote(500, 0, 0)
    r.update({"max_local_prefill_length": 100})
    assert r.prefill_remote(500, 0, 0)


_BENCH_ARGS = ["--cpu", "--model", "tiny", "--isl", "200", "--osl", "8", "--concurrency", "4", "--steps", "4",
               "--warmup", "1", "--iters-per-step", "5", "--block-size", "16", "--num-gpu-blocks", "400",
               "--max-local-prefill", "50"]


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_json(cmd, port=None, **extra_env):
    import json

    env = dict(os.environ, DX_DUMP_AFTER="200", OMP_NUM_THREADS="1", **extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    if port:
        env["MASTER_PORT"] = str(port)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4])
def test_xpyd_bench_cpu(world):
    """bench.py's N > 1 path (the driver's scaling runs) on CPU/gloo under
    torchrun: 1P1D and 2P2D, i.e. also cross pairs (prefill rank p serving
    decode rank d != p)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world)] + _BENCH_ARGS
    res = _bench_json(cmd)
    assert res["n_gpus"] == world and res["value"] > 0
    cfg = res["config"]
    assert cfg["remote_prefills"] > 0
    label = f"disagg-{world // 2}P(tp1){world - world // 2}D(tp1)"
    assert cfg["parallelism"] == label and res["metric"].endswith(label)
    assert res["ttft_p50_ms_at_qps"] is not None and res["qps"] > 0
    assert cfg["comm_world"] == world and cfg["kv_transport"] == "gloo"
    # one bench step = iters_per_step iterations of every decode rank
    assert cfg["engine_iters"] == 4 * 5 * (world - world // 2)
    # self-validating: exact collective / KV checks + token verification ran
    pf = cfg["preflight"]
    assert pf["ok"] and pf["kv_pairs_checked"] == (world // 2) * (world - world // 2)
    v = cfg["verify"]
    assert v["requests"] == 2 * (world - world // 2) and v["diverged"] == 0 and v["identical"] >= 1
    pol = cfg["disagg_policy"]
    assert (pol["mode"], pol["max_local_prefill"], pol["max_prefill_queue"]) == ("conditional", 50, 4 * (world // 2))


def test_bench_preflight_catches_corrupt_kv_piece_cpu():
    """A damaged KV piece (fault kv_transfer.corrupt_pieces) fails the
    preflight: exit status 3, no throughput line."""
    env = dict(os.environ, DX_DUMP_AFTER="200", OMP_NUM_THREADS="1", DX_FAULTS="kv_transfer.corrupt_pieces=1",
               MASTER_PORT=str(_free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + _BENCH_ARGS,
                       capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert "PREFLIGHT FAILED" in p.stderr
    assert not any(l.startswith('{"metric"') for l in p.stdout.splitlines())


def test_bench_always_remote_policy_cpu():
    """--disagg-policy always: every prompt is prefilled on a prefill engine
    (the reference benchmark's conditional-disagg: false)."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--disagg-policy", "always",
                       "--verify-tokens", "0"] + _BENCH_ARGS, port=_free_port())
    cfg = res["config"]
    assert cfg["disagg_policy"]["mode"] == "always-remote"
    assert cfg["local_prefills"] == 0 and cfg["remote_prefills"] > 0 and "verify" not in cfg


def test_bench_self_launch_cpu():
    """`bench.py --gpus 4` with no launcher spawns the 4 ranks itself (the
    verdict's 'done when': n_gpus 4, a 4-rank communicator, disagg parallelism)."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"] + _BENCH_ARGS,
                      port=_free_port())
    assert res["n_gpus"] == 4 and res["value"] > 0
    assert res["config"]["comm_world"] == 4
    assert res["config"]["parallelism"] == "disagg-2P(tp1)2D(tp1)"
    assert res["steps"] == 4 and res["warmup"] == 1


def test_bench_open_loop_cpu():
    """Fixed-QPS (open loop, Poisson) mode of the aggregated bench."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--qps", "20"] + _BENCH_ARGS)
    assert res["n_gpus"] == 1 and res["config"]["load"].startswith("open-loop")
    assert res["ttft_p50_ms"] is not None and res["config"]["engine_iters"] == 20


def test_bench_aggregated_reports_fixed_qps_ttft_cpu():
    """The driver's command shape (closed loop): after the timed window an
    open-loop Poisson segment at 80 % of the closed-loop request rate gives
    TTFT at fixed QPS in the same JSON line, and the metric names the
    aggregated layout (no disagg claim)."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py")] + _BENCH_ARGS + ["--qps-seconds", "4"])
    assert res["config"]["parallelism"] == "agg-tp1"
    assert "aggregated" in res["metric"] and "disagg" not in res["metric"]
    assert res["qps"] > 0 and res["ttft_p50_ms_at_qps"] is not None and res["requests_at_qps"] > 0


def test_disagg_refuses_silent_host_staging():
    """A GPU run with fewer devices than ranks must not silently fall back to
    gloo host staging (it reports an error unless --p2p-backend gloo)."""
    from dynamo_exp_amd.disagg import bench_disagg

    assert bench_disagg.choose_transport(torch.device("cpu"), 4, "nccl") == "gloo"


def test_serving_workers_remote_prefill_cpu():
    """LLMWorker (decode, remote_prefill) + PrefillWorker over the control plane
    prefill queue and a standalone gloo pair group: same tokens as aggregated."""
    import asyncio

    from dynamo_exp_amd.llm.workers import LLMWorker, PrefillWorker, parse_worker_args
    from dynamo_exp_amd.runtime import BackgroundServer, Context, DistributedRuntime

    cp = BackgroundServer().start()
    argv = ["--model", "tiny", "--block-size", "16", "--max-model-len", "512", "--num-gpu-blocks", "300",
            "--device", "cpu", "--max-local-prefill-length", "10", "--max-prefill-queue-size", "100"]
    prompt = list(range(30, 30 + 120))
    agg = _engine()
    ref = _run(agg, "ref", prompt, 8)

    async def main():
        drt = await DistributedRuntime.create(cp.address)
        comp = drt.namespace("dx").component("Worker")
        dw = await LLMWorker(parse_worker_args(argv + ["--remote-prefill"]), drt, comp, drt.primary_lease,
                             "dx").start()
        dw.engine.model = agg.model
        dw.engine.runner.model = agg.model
        drt2 = await DistributedRuntime.create(cp.address)
        pw = await PrefillWorker(parse_worker_args(argv), drt2, drt2.namespace("dx").component("PrefillWorker"),
                                 drt2.primary_lease, "dx").start()
        pw.engine.model = agg.model
        pw.engine.runner.model = agg.model
        ptask = asyncio.create_task(pw.run())
        req = {"token_ids": prompt, "stop_conditions": {"max_tokens": 8, "ignore_eos": True},
               "sampling_options": {}, "eos_token_ids": [2]}
        toks = []
        async for out in dw.generate(req, Context()):
            toks += out["token_ids"]
        assert dw.agent.stats["recv"] == 1 and pw.agent.stats["sent"] == 1
        await drt2.primary_lease.revoke()
        await asyncio.wait_for(ptask, 10)
        dw.shutdown()
        pw.shutdown()
        await drt.close(1)
        await drt2.close(1)
        return toks

    try:
        toks = asyncio.run(asyncio.wait_for(main(), 120))
    finally:
        cp.stop()
    assert toks == ref


@pytest.mark.parametrize("ptp,dtp", [(1, 2), (1, 4), (2, 1), (2, 4), (4, 2)])
def test_tp_relayout_between_prefill_and_decode(ptp, dtp):
    """P->D KV relayout when prefill and decode TP differ (K4/K6 semantics)."""
    from dynamo_exp_amd.disagg.transfer import tp_relayout_plan

    L, NB, H, BS, D = 2, 6, 8, 16, 8
    full = torch.randn(L, 2, NB, H, BS, D).to(torch.bfloat16)
    src = [full[:, :, :, r * (H // ptp):(r + 1) * (H // ptp)].contiguous() for r in range(ptp)]
    dst = [torch.zeros(L, 2, NB, H // dtp, BS, D, dtype=torch.bfloat16) for _ in range(dtp)]
    blocks_p, blocks_d = [1, 4, 2], [5, 0, 3]
    for pc in tp_relayout_plan(ptp, dtp, H, BS, D):
        buf = pack_blocks(src[pc.src_rank], blocks_p, inner_off=pc.src_inner_off, inner_bytes=pc.nbytes)
        unpack_blocks(dst[pc.dst_rank], buf, blocks_d, inner_off=pc.dst_inner_off, inner_bytes=pc.nbytes)
    for r in range(dtp):
        want = full[:, :, blocks_p, r * (H // dtp):(r + 1) * (H // dtp)]
        assert torch.equal(dst[r][:, :, blocks_d], want)


def test_prefill_pulls_decode_prefix_instead_of_recomputing():
    """READ path (reference Patch:1296-1360 read_blocks): the decode engine
    caches 64 of the prompt's tokens, the prefill engine none; the prefill
    engine parks the request, pulls those 4 blocks, computes only the other
    ISL - 64 tokens, and the decode output equals the aggregated engine's."""
    agg = _engine()
    prompt = list(range(40, 40 + 150))
    ref = _run(agg, "a", prompt, 10)
    prefill = _engine(model=agg.model)
    decode = _engine(model=agg.model)
    _run(decode, "warm", prompt[:64] + [9] * 10, 2)

    got = []
    decode.add_request("x", prompt, SamplingParams(max_tokens=10, ignore_eos=True),
                       on_output=lambda r, t, lp, fin: got.extend(t), remote_prefill=True)
    decode.step()
    dreq = decode.scheduler.remote["x"]
    skip = dreq.num_computed // 16
    assert skip == 4

    reads = []
    prefill.scheduler.on_remote_read = lambda r, first, last: reads.append((r, first, last))
    sent = {}
    prefill.prefill_done_hook = lambda r: sent.setdefault("req", r)
    prefill.add_request("x", prompt, SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True,
                        remote_read_blocks=skip)
    prefill.step()  # admits, parks in READING (nothing to compute yet)
    assert len(reads) == 1 and "req" not in sent
    preq, first, last = reads[0]
    assert (first, last) == (0, 4) and "x" in prefill.scheduler.reading
    # "the wire": decode serves blocks [first, last) of its request
    buf = pack_blocks(decode.runner.kv_cache, dreq.block_ids[first:last])
    unpack_blocks(prefill.runner.kv_cache, buf, preq.block_ids[first:last])
    prefill.finish_remote_read("x")
    t0 = prefill.runner.timing["prefill_tokens"]
    while "req" not in sent:
        prefill.step()
    assert prefill.runner.timing["prefill_tokens"] - t0 == len(prompt) - 64  # the prefix was not recomputed
    nblk = (len(prompt) + 15) // 16
    buf = pack_blocks(prefill.runner.kv_cache, preq.block_ids[skip:nblk])
    unpack_blocks(decode.runner.kv_cache, buf, dreq.block_ids[skip:nblk])
    prefill.finish_transfer("x")
    decode.finish_remote_prefill("x", preq.output[0], preq.logprobs[0])
    while decode.has_unfinished():
        decode.step()
    assert got == ref
    # the pulled blocks are now in the prefill engine's own prefix cache
    assert prefill.kv.prefix_hit_tokens_for(prompt) >= 64


def test_abort_during_prefix_read_drains_without_unpacking():
    """a request aborted while its prefix pull is in flight
    has freed its blocks; when the pull lands the agent must only drain it
    (no unpack into blocks that may belong to another request) and must not
    resume the request."""
    from dynamo_exp_amd.disagg.agent import KVTransferAgent

    prefill = _engine()
    prompt = list(range(40, 40 + 150))
    reads = []
    prefill.scheduler.on_remote_read = lambda r, first, last: reads.append((r, first, last))
    prefill.add_request("x", prompt, SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True,
                        remote_read_blocks=4)
    prefill.step()
    assert reads and "x" in prefill.scheduler.reading

    class _DP:  # the data plane's side of finish_read, recorded
        calls = []

        def finish_read(self, rid, unpack):
            self.calls.append((rid, unpack))
            return True

    agent = KVTransferAgent.__new__(KVTransferAgent)
    agent.engine, agent.dp = prefill, _DP()
    agent._read1 = {}
    resumed = []
    real = prefill.finish_remote_read
    prefill.finish_remote_read = lambda rid, ok=True: (resumed.append((rid, ok)), real(rid, ok))
    prefill.abort("x")
    assert "x" not in prefill.scheduler.reading
    agent.finish_read({"rid": "x", "ok": True})
    assert _DP.calls == [("x", False)] and resumed == []
    # a live read still unpacks and resumes
    prefill.add_request("y", prompt, SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True,
                        remote_read_blocks=4)
    prefill.step()
    agent.finish_read({"rid": "y", "ok": True})
    assert _DP.calls[-1] == ("y", True) and resumed == [("y", True)]
    assert prefill.requests["y"].num_computed == 64
    # a READ served after the decode engine gave the request up
    # (verdict false: filler bytes) is drained, never registered, and the
    # request recomputes its prefix
    prompt2 = list(range(300, 300 + 150))
    prefill.add_request("z", prompt2, SamplingParams(max_tokens=1, ignore_eos=True), remote_decode=True,
                        remote_read_blocks=4)
    prefill.step()
    assert "z" in prefill.scheduler.reading
    agent.finish_read({"rid": "z", "ok": False})
    assert _DP.calls[-1] == ("z", False) and resumed[-1] == ("z", False)
    z = prefill.requests["z"]
    assert z.num_computed == 0 and z.remote_read_blocks == 0 and "z" not in prefill.scheduler.reading
    assert prefill.kv.prefix_hit_tokens_for(prompt2) == 0  # nothing of z was registered
    t0 = prefill.runner.timing["prefill_tokens"]
    prefill.step()
    assert prefill.runner.timing["prefill_tokens"] - t0 == len(prompt2)  # the whole prompt is computed


def _xfer_worker(rank, port, q):
    import torch.distributed as dist

    from dynamo_exp_amd.disagg.transfer import KVDataPlane, WorldLinks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    rev = dist.new_group(backend="gloo")
    torch.manual_seed(rank)
    L, NB, H, BS, D = 6, 12, 2, 16, 8
    kv = torch.randn(L, 2, NB, H, BS, D).to(torch.bfloat16)
    links = WorldLinks({"p": [0], "d": [1]}, group=dist.group.WORLD, rev_group=rev)
    x = KVDataPlane(kv, links, layer_group_count=3, pool_cap_bytes=64 << 20)
    out = {}
    if rank == 0:  # prefill: stream two requests of different sizes in one forward, then pull [2, 5]
        anns = [x.begin_send("r", [3, 7, 1], "d"), x.begin_send("s", [10, 11], "d")]
        for layer in range(L):
            x.on_layer(layer)  # packs + sends a group of both requests at layers 1, 3, 5 (group-major)
        x.end_forward()
        dist.broadcast_object_list([anns], src=0)
        done = set()
        while len(done) < 2:
            done.update(x.poll_sends())
        x.post_read("p", [8, 9], "d")
        while not x.reads_landed():
            pass
        assert x.finish_read("p")
        out["pulled"] = kv[:, :, [8, 9]].clone()
        out["sent"] = kv[:, :, [3, 7, 1, 10, 11]].clone()
        out["groups"] = len(x.groups)
        out["pool"] = dict(x.pool.stats)
    else:  # decode: receive into blocks [0, 4, 6] / [7, 3]; serve blocks [2, 5] to the read
        obj = [None]
        dist.broadcast_object_list(obj, src=0)
        a, b = obj[0]
        x.post_recv_batch("p", 1, [("r", a["nblocks"], [0, 4, 6]), ("s", b["nblocks"], [7, 3])])
        landed = set()
        while len(landed) < 2:
            landed.update(x.recvs_landed())
        assert x.finish_recv("r") and x.finish_recv("s")
        x.serve_read("p", [2, 5], "p")
        while x.poll_served():
            pass
        out["recv"] = kv[:, :, [0, 4, 6, 7, 3]].clone()
        out["served"] = kv[:, :, [2, 5]].clone()
    # by value: a torch tensor in a multiprocessing queue travels as a shared-
    # memory fd the parent fetches from this process later -- racing its exit
    out = {k: (v.float().numpy() if torch.is_tensor(v) else v) for k, v in out.items()}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_kv_transfer_layer_streamed_and_read_two_processes():
    """KVDataPlane over a real 2-process group (gloo standing in for RCCL):
    layer-group streamed WRITE into other block ids, READ in the reverse
    direction on its own group, pooled staging reused."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xfer_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert (res[1]["recv"] == res[0]["sent"]).all()
    assert (res[0]["pulled"] == res[1]["served"]).all()
    assert res[0]["groups"] == 3


def test_staging_pool_reservations():
    """Backpressure bookkeeping: reservations count against the cap, an idle
    pool admits one oversized transfer, take/give recycle size classes."""
    from dynamo_exp_amd.disagg.transfer import StagingPool

    p = StagingPool("cpu", cap_bytes=32 << 20, granule=8 << 20)
    assert p.reserve(5 << 20, 9 << 20)  # 8 + 16 MiB classes
    assert not p.reserve(9 << 20)  # 24 + 16 > 32
    assert p.stats["deferred"] == 1
    p.unreserve(5 << 20)
    a = p.take(5 << 20)
    p.unreserve(9 << 20)
    b = p.take(9 << 20)
    assert p.in_use == 24 << 20 and p.reserved == 0 and p.stats["over_cap"] == 0
    p.give(a)
    p.give(b)
    assert p.reserve(40 << 20)  # idle pool: one transfer above the cap still goes through
    assert not p.reserve(1)
    p.unreserve(40 << 20)
    c = p.take(5 << 20)
    assert c.numel() == 8 << 20 and p.stats["reuses"] == 1


def test_serving_workers_prefix_read_cpu():
    """Serving-worker READ path: the decode worker caches a 64-token prefix
    (served locally), the prefill worker does not; the next long request with
    that prefix goes remote, the prefill worker pulls the 4 cached blocks over
    the reverse pair group and computes only the other 56 tokens."""
    import asyncio

    from dynamo_exp_amd.llm.workers import LLMWorker, PrefillWorker, parse_worker_args
    from dynamo_exp_amd.runtime import BackgroundServer, Context, DistributedRuntime

    cp = BackgroundServer().start()
    argv = ["--model", "tiny", "--block-size", "16", "--max-model-len", "512", "--num-gpu-blocks", "300",
            "--device", "cpu", "--max-local-prefill-length", "70", "--max-prefill-queue-size", "100",
            "--min-read-tokens", "32"]
    prefix = list(range(300, 364))
    warm = prefix + [5, 6]
    prompt = prefix + list(range(400, 456))
    agg = _engine()
    ref = _run(agg, "ref", prompt, 6)

    async def main():
        drt = await DistributedRuntime.create(cp.address)
        dw = await LLMWorker(parse_worker_args(argv + ["--remote-prefill", "--conditional-disagg"]), drt,
                             drt.namespace("dx").component("Worker"), drt.primary_lease, "dx").start()
        dw.engine.model = agg.model
        dw.engine.runner.model = agg.model
        drt2 = await DistributedRuntime.create(cp.address)
        pw = await PrefillWorker(parse_worker_args(argv), drt2, drt2.namespace("dx").component("PrefillWorker"),
                                 drt2.primary_lease, "dx").start()
        pw.engine.model = agg.model
        pw.engine.runner.model = agg.model
        ptask = asyncio.create_task(pw.run())

        async def gen(p, n):
            req = {"token_ids": p, "stop_conditions": {"max_tokens": n, "ignore_eos": True},
                   "sampling_options": {}, "eos_token_ids": [2]}
            toks = []
            async for out in dw.generate(req, Context()):
                toks += out["token_ids"]
            return toks

        await gen(warm, 2)  # local prefill: the decode worker now caches the prefix
        toks = await gen(prompt, 6)
        stats = dict(pw.agent.stats), dict(dw.agent.stats), pw.engine.runner.timing["prefill_tokens"]
        await drt2.primary_lease.revoke()
        await asyncio.wait_for(ptask, 10)
        dw.shutdown()
        pw.shutdown()
        await drt.close(1)
        await drt2.close(1)
        return toks, stats

    try:
        toks, (pst, dst, ptoks) = asyncio.run(asyncio.wait_for(main(), 120))
    finally:
        cp.stop()
    assert pst["reads"] == 1 and dst["served"] == 1 and pst["sent"] == 1
    assert ptoks == len(prompt) - len(prefix)
    assert toks == ref


def test_bench_python_control_plane_fallback_cpu():
    """Without the native server (DX_CTRLD=python) rank 0 hosts the asyncio
    control plane on a thread; the port still reaches the other ranks over
    the gloo group."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + _BENCH_ARGS,
                      port=_free_port(), DX_CTRLD="python")
    assert res["n_gpus"] == 2 and res["value"] > 0 and res["config"]["comm_world"] == 2


@pytest.mark.slow
@pytest.mark.parametrize("layout,label", [
    (["--gpus", "4", "--tp", "2"], "disagg-1P(tp2)1D(tp2)"),
    (["--gpus", "5", "--prefill-tp", "1", "--decode-tp", "4", "--prefill-ranks", "1"], "disagg-1P(tp1)1D(tp4)"),
    (["--gpus", "3", "--prefill-tp", "2", "--decode-tp", "1", "--prefill-ranks", "2"], "disagg-1P(tp2)1D(tp1)"),
])
def test_bench_tp_disagg_layouts_cpu(layout, label):
    """bench.py with TP engines (verdict r2 #1): 1P1D at TP2, the reference's
    asymmetric layout (prefill TP1 -> decode TP4: one replicated KV head per
    decode rank) and prefill TP2 -> decode TP1.  Every rank joins the
    N-rank communicator, the KV moves as relayout pieces over the one data
    plane, and fixed prompts decode exactly the tokens of a TP1 aggregated
    engine on the same weights."""
    args = ["--cpu", "--model", "tiny", "--isl", "200", "--osl", "8", "--concurrency", "4", "--steps", "2",
            "--warmup", "1", "--iters-per-step", "5", "--block-size", "16", "--num-gpu-blocks", "400",
            "--max-local-prefill", "50", "--qps-segment", "0", "--verify-tokens", "3"]
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py")] + layout + args, port=_free_port())
    cfg = res["config"]
    assert cfg["parallelism"] == label and cfg["comm_world"] == int(layout[1])
    assert cfg["verify"] == {"requests": 3, "identical": 3, "near_tie": 0, "diverged": 0}, cfg.get("verify")
    assert cfg["remote_prefills"] > 0 and cfg["kv_transfer_GB"] >= 0
    # preflight: every TP group's collectives checked exactly, the relayout pieces moved byte-exact
    pf = cfg["preflight"]
    n_tp = sum(1 for t in (cfg["prefill_tp"], cfg["decode_tp"]) if t > 1)
    assert pf["ok"] and pf["kv_pairs_checked"] == 1 and pf["tp_groups_checked"] == n_tp


_N8_ARGS = ["--cpu", "--model", "tiny", "--isl", "200", "--osl", "8", "--concurrency", "2", "--steps", "2",
            "--warmup", "1", "--iters-per-step", "4", "--block-size", "16", "--num-gpu-blocks", "300",
            "--max-local-prefill", "50", "--qps-segment", "0", "--verify-tokens", "2"]


@pytest.mark.slow
@pytest.mark.parametrize("layout,label,n_pre,n_dec,n_tp", [
    (["--gpus", "8"], "disagg-4P(tp1)4D(tp1)", 4, 4, 0),
    (["--gpus", "8", "--tp", "4"], "disagg-1P(tp4)1D(tp4)", 1, 1, 2),
    (["--gpus", "8", "--prefill-tp", "1", "--decode-tp", "4", "--prefill-ranks", "4"], "disagg-4P(tp1)1D(tp4)",
     4, 1, 1),
    # the reference benchmark's precision on that layout (disagg.yaml:16-59): w8a8 fp8 + fp8 KV cache, the
    # prefill ranks sized by their own memory flag
    (["--gpus", "8", "--prefill-tp", "1", "--decode-tp", "4", "--prefill-ranks", "4", "--quantization", "fp8",
      "--kv-cache-dtype", "fp8", "--prefill-gpu-mem-util", "0.9"], "disagg-4P(tp1)1D(tp4)", 4, 1, 1),
])
def test_bench_n8_layouts_cpu(layout, label, n_pre, n_dec, n_tp):
    """the layouts of the driver's N = 8 run and of
    config 4 (reference examples/llm/benchmarks/disagg.yaml:45-56: 4 prefill
    TP1 workers + 1 decode TP4 worker) at world 8 on CPU/gloo -- the exact
    group-creation order, the 16-pair link warm-up of 4P4D, the preflight's
    pair and TP-group counts and the token verification."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py")] + layout + _N8_ARGS, port=_free_port())
    cfg = res["config"]
    assert res["n_gpus"] == 8 and cfg["parallelism"] == label and cfg["comm_world"] == 8
    pf = cfg["preflight"]
    assert pf["ok"] and pf["kv_pairs_checked"] == n_pre * n_dec and pf["tp_groups_checked"] == n_tp, pf
    v = cfg["verify"]
    assert v["diverged"] == 0 and v["requests"] == 2 * n_dec, v
    assert cfg["remote_prefills"] > 0 and res["value"] > 0


@pytest.mark.slow
def test_bench_n8_preflight_catches_corrupt_piece_cpu():
    """At world 8 (4P(tp1)1D(tp4): relayout pieces to four decode ranks) one
    damaged KV piece fails the preflight: the ranks exit 3, no throughput line."""
    env = dict(os.environ, DX_DUMP_AFTER="250", OMP_NUM_THREADS="1", DX_FAULTS="kv_transfer.corrupt_pieces=1",
               MASTER_PORT=str(_free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--prefill-tp", "1",
                        "--decode-tp", "4", "--prefill-ranks", "4"] + _N8_ARGS,
                       capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode != 0, p.stderr[-3000:]  # ranks exit 3; the launcher reports 1
    assert "PREFLIGHT FAILED" in p.stderr and "exitcode  : 3" in p.stderr
    assert not any(l.startswith('{"metric"') for l in p.stdout.splitlines())


def test_bench_staging_backpressure_cpu():
    """Staging backpressure (verdict r2 weak #10): a 16 MiB pool per rank
    (two 8 MiB transfers) under 64 closed-loop streams, every prompt remote:
    transfers wait for staging (deferred > 0), the pool never goes over its
    cap, and the run completes."""
    args = ["--cpu", "--model", "tiny", "--isl", "200", "--osl", "8", "--concurrency", "32", "--steps", "2",
            "--warmup", "1", "--iters-per-step", "5", "--block-size", "16", "--num-gpu-blocks", "1200",
            "--max-local-prefill", "50", "--max-prefill-queue", "1000", "--qps-segment", "0",
            "--staging-bytes", str(16 << 20)]
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args, port=_free_port())
    cfg = res["config"]
    assert cfg["staging_over_cap"] == 0
    assert cfg["staging_deferred"] > 0
    assert cfg["remote_prefills"] >= 64


@pytest.mark.slow
def test_bench_aggregated_data_parallel_cpu():
    """`--mode agg`: N/TP aggregated TP engines on the node (the same-node
    aggregated baseline of the scaling curve), windows merged over leaders."""
    args = ["--cpu", "--model", "tiny", "--isl", "200", "--osl", "8", "--concurrency", "4", "--steps", "2",
            "--warmup", "1", "--iters-per-step", "5", "--block-size", "16", "--num-gpu-blocks", "400",
            "--qps-seconds", "2"]
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--mode", "agg", "--tp", "2"]
                      + args, port=_free_port())
    cfg = res["config"]
    assert cfg["parallelism"] == "agg-dp2-tp2" and cfg["comm_world"] == 4 and res["value"] > 0
    assert cfg["engine_iters"] == 2 * 2 * 5  # two engines x steps x iters_per_step


def test_bench_concurrency_sweep_cpu():
    """--sweep: the reference's concurrency sweep (perf.sh:17-54) on one
    engine -- one point per concurrency with tok/s/GPU and tok/s/user."""
    # a longer window per point (last flag wins) so batching shows through CPU timing noise
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--sweep", "1,4"] + _BENCH_ARGS
                      + ["--iters-per-step", "12"])
    pts = res["points"]
    assert [p["concurrency"] for p in pts] == [1, 4]
    assert all(p["tok_s_gpu"] > 0 and p["tok_s_user"] and p["ttft_p50_ms"] is not None for p in pts)
    assert pts[1]["tok_s_gpu"] > pts[0]["tok_s_gpu"]  # batching raises throughput per GPU


def test_bench_disagg_concurrency_sweep_cpu():
    """--sweep with N > 1: the same per-GPU concurrency points through the
    1P1D layout's engines (gloo), one JSON line of points with tok/s/GPU
    (node output / N) vs tok/s/user -- the reference's agg-vs-disagg method."""
    res = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--sweep", "1,4"]
                      + _BENCH_ARGS)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "disagg-1P(tp1)1D(tp1)"
    pts = res["points"]
    assert [p["concurrency_per_gpu"] for p in pts] == [1, 4]
    assert all(p["tok_s_gpu"] > 0 and p["tok_s_user"] for p in pts), pts
    assert res["config"]["remote_prefills"] > 0 and res["config"]["preflight"]["ok"], res["config"]


def test_remote_prefill_falls_back_to_local_when_transfer_never_starts():
    """Failure handling: a remote prefill whose KV transfer never
    started -- the prefill worker dropped it ("fail" notification) or went
    silent past the start timeout -- is prefilled on the decode engine
    itself, with the tokens an aggregated engine produces; a request whose
    announcement arrived is never taken back (its receives are posted)."""
    import time

    from dynamo_exp_amd.disagg.agent import KVTransferAgent, decode_leader_hook, install_decode
    from dynamo_exp_amd.disagg.transfer import LoopbackHub, LoopbackLinks
    from dynamo_exp_amd.parallel.tp import ReplicatedEngine

    kw = dict(model="tiny", device="cpu", block_size=16, max_model_len=256, num_gpu_blocks=64, max_num_seqs=4,
              use_cuda_graph=False)
    ref = LLMEngine(EngineConfig(**kw))
    prompts = [list(range(5 + i, 60 + 3 * i)) for i in range(3)]
    want = []
    for i, p in enumerate(prompts):
        toks = []
        ref.add_request(f"a{i}", p, SamplingParams(max_tokens=5, ignore_eos=True),
                        on_output=lambda r, t, lp, fin, toks=toks: toks.extend(t))
        while ref.has_unfinished():
            ref.step()
        want.append(toks)
    eng = LLMEngine(EngineConfig(**kw), model=ref.model)
    rep = ReplicatedEngine(eng, None, 0, 1)
    class _Rec:  # the control plane: records what the agent publishes
        sent = []

        def fire(self, op, subject, data):
            import msgpack

            self.sent.append((subject, msgpack.unpackb(data, raw=False)))

    agent = KVTransferAgent(eng, _Rec(), "d", "t", links=LoopbackLinks(LoopbackHub("cpu"), "d"))
    install_decode(rep, agent)
    hook = decode_leader_hook(rep, agent, start_timeout=0.3)
    got = {}

    def add(i):
        got[i] = []
        rep.add_request(f"r{i}", prompts[i], SamplingParams(max_tokens=5, ignore_eos=True),
                        on_output=lambda r, t, lp, fin: got[i].extend(t), remote_prefill=True)

    for i in range(3):
        add(i)
    rep.step()
    assert set(eng.scheduler.remote) == {"r0", "r1", "r2"}
    agent.inbox.append({"t": "fail", "rid": "r0"})  # dropped by the prefill worker before its WRITE
    agent.inbox.append({"t": "start", "src": "p", "src_tp": 1, "reqs": [{"rid": "r2", "nblocks": 4}]})
    hook()
    rep.step()
    assert "r0" not in eng.scheduler.remote and {"r1", "r2"} <= set(eng.scheduler.remote)
    time.sleep(0.35)  # r1: no announcement within the timeout
    t0 = time.time()
    while "r1" in eng.scheduler.remote and time.time() - t0 < 5:
        hook()
        rep.step()
    assert "r1" not in eng.scheduler.remote
    assert "r2" in eng.scheduler.remote  # announced: its transfer is in flight, never taken back
    while any(len(got[i]) < 5 for i in (0, 1)):
        hook()
        rep.step()
    assert [got[0], got[1]] == want[:2]
    assert agent.stats["fallbacks"] == 2 and eng.scheduler.fallbacks == 2
    # each fallback cancels the queued prompt for the prefill workers
    assert sorted(m["rid"] for s, m in _Rec.sent if s == "kv_wire.t" and m["t"] == "cancel") == ["r0", "r1"]


def test_staging_buffers_taken_in_inference_mode_stay_writable():
    """A staging buffer first taken inside inference mode (the preflight, a
    forward's layer hook) and recycled must accept in-place writes from the
    transfer handlers, which run outside it (the 70B@20 rehearsal's serve_read
    failed on an inference tensor, round 5)."""
    from dynamo_exp_amd.disagg.transfer import StagingPool

    pool = StagingPool("cpu", 64 << 20)
    with torch.inference_mode():
        b = pool.take(1 << 20)
    pool.give(b)
    b2 = pool.take(1 << 20)
    assert b2.data_ptr() == b.data_ptr() and not b2.is_inference()
    b2[:16].copy_(torch.arange(16, dtype=torch.uint8))
