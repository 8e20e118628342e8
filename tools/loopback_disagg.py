#!/usr/bin/env python3
"""One-GPU measurement of the device KV data plane (disagg/loopback.py).

A prefill engine and a decode engine share one MI355X; prompts go through
the production transfer path (layer-streamed WRITE on the copy stream,
device staging, unpack) over LoopbackLinks.  Reports, for prefill batches:

* host enqueue time of the prefill launch (`runner.launch`, which runs the
  forward and its layer hooks): without a host sync inside the hooks it is a
  small fraction of the batch's GPU time; a sync at every layer-group
  boundary would make it track the GPU time;
* GPU time of the prefill forwards with the transfer vs the same batches on
  the same engine with no transfer (copy-stream packs overlap the forward);
* KV bytes moved and the transfer latency from announcement to unpack.

    python tools/loopback_disagg.py --prompts 40 --out profiles/r4_loopback_1p1d.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--prompts", type=int, default=40)
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=16)
    ap.add_argument("--batch-tokens", type=int, default=16384)
    ap.add_argument("--groups", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    from dynamo_exp_amd.bench.serving import PromptGen
    from dynamo_exp_amd.disagg.loopback import Loopback1P1D
    from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
    from dynamo_exp_amd.engine.request import SamplingParams

    dev = "cuda:0"
    nblk = a.prompts * ((a.isl + a.osl) // 64 + 2) + 64
    kw = dict(model=a.model, device=dev, block_size=64, max_model_len=a.isl + a.osl + 64, num_gpu_blocks=nblk, seed=1)
    pe = LLMEngine(EngineConfig(max_num_seqs=32, use_cuda_graph=False, chunked_prefill=False,
                                max_num_batched_tokens=a.batch_tokens, **kw))
    de = LLMEngine(EngineConfig(max_num_seqs=max(8, a.prompts), graph_sizes=(1, 2, 4, 8, 16, 32, 64),
                                max_num_batched_tokens=8192, **kw), model=pe.model)
    pe.warmup()
    de.warmup()
    gen = PromptGen(7, a.isl, pe.model_cfg.vocab_size)

    launch_t: list[tuple] = []
    orig_launch = pe.runner.launch

    def timed_launch(batch, prev=None):
        t0 = time.perf_counter()
        h = orig_launch(batch, prev)
        launch_t.append((time.perf_counter() - t0, batch.kind, sum(batch.num_new)))
        return h

    pe.runner.launch = timed_launch

    def gpu_s(eng):
        eng.runner.harvest_gpu_time()
        return eng.runner.timing["prefill_gpu"]

    # ---- A: the same engine, prefill only, no transfer
    torch.cuda.synchronize()
    g0, t0 = gpu_s(pe), time.perf_counter()
    for i in range(a.prompts):
        pe.add_request(f"a{i}", gen(), SamplingParams(max_tokens=1, ignore_eos=True))
    while pe.has_unfinished():
        pe.step()
    torch.cuda.synchronize()
    base = {"wall_s": time.perf_counter() - t0, "gpu_s": gpu_s(pe) - g0, "launches": list(launch_t)}
    pe.kv.reset_prefix_cache()
    launch_t.clear()

    # ---- B: 1P1D over the loopback data plane
    lb = Loopback1P1D(pe, de, pool_cap_bytes=16 << 30, layer_group_count=a.groups)
    done = {}
    torch.cuda.synchronize()
    g0, t0 = gpu_s(pe), time.perf_counter()
    for i in range(a.prompts):
        lb.add(f"b{i}", gen(), SamplingParams(max_tokens=a.osl, ignore_eos=True),
               on_output=lambda r, t, lp, fin: done.__setitem__(r.request_id, fin) if fin else None, remote=True)
    lb.run_until_idle(900)
    torch.cuda.synchronize()
    xfer = {"wall_s": time.perf_counter() - t0, "gpu_s": gpu_s(pe) - g0, "launches": list(launch_t)}

    def summ(d):
        pre = [(t, n) for t, k, n in d["launches"] if k == "prefill"]
        return {"wall_s": round(d["wall_s"], 3), "prefill_gpu_s": round(d["gpu_s"], 3),
                "prefill_batches": len(pre), "prefill_tokens": sum(n for _, n in pre),
                "launch_host_ms_mean": round(1e3 * sum(t for t, _ in pre) / max(1, len(pre)), 2),
                "launch_host_ms_max": round(1e3 * max((t for t, _ in pre), default=0), 2),
                "gpu_ms_per_batch": round(1e3 * d["gpu_s"] / max(1, len(pre)), 2)}

    out = {"model": a.model, "isl": a.isl, "prompts": a.prompts, "layer_groups": a.groups,
           "no_transfer": summ(base), "loopback_1p1d": summ(xfer), "completed": len(done),
           "kv_sent_GB": round(lb.pa.dp.stats["sent_bytes"] / 1e9, 3),
           "kv_recv_GB": round(lb.da.dp.stats["recv_bytes"] / 1e9, 3),
           "hub": lb.hub.stats, "prefill_send_time_s": round(lb.pa.dp.stats["send_time"], 3),
           "decode_recv_time_s": round(lb.da.dp.stats["recv_time"], 3),
           "staging_peak_GB": round(lb.pa.pool.stats["peak"] / 1e9, 2)}
    b, x = out["no_transfer"], out["loopback_1p1d"]
    out["gpu_time_ratio"] = round(x["prefill_gpu_s"] / max(1e-9, b["prefill_gpu_s"]), 3)
    out["launch_host_over_gpu"] = round(x["launch_host_ms_mean"] / max(1e-9, x["gpu_ms_per_batch"]), 3)
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
