"""Pre-flight checks of a multi-GPU bench run: before the
timed window, prove that the collectives and the KV data plane of THIS
layout move the right bytes, so a throughput number from random weights and
ignore_eos cannot hide a broken cross-GPU path.

* `tp_check` (every TP group): the custom xGMI all-reduce one-shot and
  two-shot, the RCCL all-reduce branch (messages above the custom buffer,
  e.g. 70B TP4 prefill at 8192 tokens), the custom all-gather, and one
  hipGraph replay of a captured all-reduce -- each against the exact sum.
  Inputs are small multiples of 1/4 in [-2, 2): every partial sum of up to
  8 ranks is exact in bf16 whatever the reduction order, so the check is
  bitwise, not a tolerance.
* `kv_check` (every (prefill engine, decode engine) pair): one WRITE of a
  byte pattern through `KVDataPlane` (pack, relayout pieces, links, unpack)
  and one READ in the reverse direction, each verified byte for byte on the
  receiving ranks.  The pattern is a function of (layer, K|V, block index in
  the transfer, GLOBAL KV head, byte), so a TP relayout that puts a head on
  the wrong rank or offset fails too.

Both return a small dict of results; `ok` is False on any mismatch.
"""
from __future__ import annotations

import time

import torch

from .transfer import kv_heads_of_rank


def _pattern(n: int, rank: int, seed: int, device) -> torch.Tensor:
    i = torch.arange(n, device=device, dtype=torch.int64)
    return ((((i * 40503 + rank * 7919 + seed) % 16) - 8).to(torch.float32) / 4).to(torch.bfloat16)


def _expected_sum(n: int, world: int, seed: int, device) -> torch.Tensor:
    acc = torch.zeros(n, device=device, dtype=torch.float32)
    for r in range(world):
        acc += _pattern(n, r, seed, device).float()
    return acc.to(torch.bfloat16)


def tp_check(tp, device) -> dict:
    """Run on every rank of a TP group (same calls in the same order)."""
    res: dict = {"tp": tp.size}
    if tp.size <= 1:
        res["ok"] = True
        return res
    t0 = time.perf_counter()
    ar = tp.custom_ar
    cases = [("one_shot", 128 * 4096), ("two_shot", 4 << 20)]
    cases.append(("rccl", (ar.max_bytes // 2 + (4 << 20)) if ar is not None else (8 << 20)))
    ok = True
    device_group = device.type == "cuda" and tp._device_collectives()
    for seed, (name, n) in enumerate(cases, 1):
        if name == "rccl" and device.type == "cuda" and not device_group:
            res[name] = {"skipped": "gloo TP group (ranks sharing one GPU): no device collective above the buffer"}
            continue
        if device.type != "cuda":
            n = min(n, 1 << 16)  # gloo rehearsal: the same code, smaller messages
        x = _pattern(n, tp.rank, seed, device)
        dist_path = "rccl" if device_group or device.type != "cuda" else "gloo"
        path = dist_path if ar is None or not ar.should_use(x) else ("custom-1" if n * 2 <= ar.one_shot_max else "custom-2")
        got = tp.all_reduce(x)
        good = bool(torch.equal(got, _expected_sum(n, tp.size, seed, device)))
        res[name] = {"elems": n, "path": path, "exact": good}
        ok &= good
    # all-gather ([B, 5] fp32 rows: the vocab-sharded sampler's partials)
    rows = _pattern(64 * 5, tp.rank, 9, device).float().view(64, 5)
    g = tp.gather_rows(rows)
    want = torch.stack([_pattern(64 * 5, r, 9, device).float().view(64, 5) for r in range(tp.size)])
    res["gather"] = bool(torch.equal(g.to(want.device), want))
    ok &= res["gather"]
    # one captured all-reduce replayed (the decode graphs' form: input in the registered buffer)
    if ar is not None and device.type == "cuda":
        shape = (64, 4096)
        buf = ar.buffer(shape)
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            ar.all_reduce(buf)  # warm outside the capture
        torch.cuda.current_stream(device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = ar.all_reduce(buf)
        good = True
        for seed in (21, 22):
            buf.copy_(_pattern(shape[0] * shape[1], tp.rank, seed, device).view(shape))
            graph.replay()
            good &= bool(torch.equal(out.view(-1), _expected_sum(shape[0] * shape[1], tp.size, seed, device)))
        res["graph_replay"] = good
        ok &= good
        del graph
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    res["ok"] = bool(ok)
    res["ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    return res


# ------------------------------------------------------------------------- KV
def _kv_bytes_pattern(kv: torch.Tensor, blocks: list[int], tp_rank: int, tp: int, total_heads: int, tag: int,
                      n_blocks: int | None = None) -> torch.Tensor:
    """Expected bytes of `blocks` ([L, 2, n, Hl, BS*D*elem] uint8) on a rank
    holding heads kv_heads_of_rank(tp_rank, tp, total_heads)."""
    L, two, NB, Hl, BS, D = kv.shape
    hb = BS * D * kv.element_size()
    h0, hn = kv_heads_of_rank(tp_rank, tp, total_heads)
    n = len(blocks) if n_blocks is None else n_blocks
    dev = kv.device
    lay = torch.arange(L, device=dev).view(L, 1, 1, 1, 1)
    kvi = torch.arange(2, device=dev).view(1, 2, 1, 1, 1)
    b = torch.arange(n, device=dev).view(1, 1, n, 1, 1)
    h = (h0 + torch.arange(hn, device=dev)).view(1, 1, 1, hn, 1)
    byte = torch.arange(hb, device=dev).view(1, 1, 1, 1, hb)
    v = lay * 31 + kvi * 17 + b * 13 + h * 7 + byte * 3 + tag * 101
    return (v % 251).to(torch.uint8)


def _fill(kv, blocks, tp_rank, tp, total_heads, tag) -> None:
    idx = torch.tensor(blocks, device=kv.device)
    L, two, NB, Hl, BS, D = kv.shape
    view = kv.view(torch.uint8).view(L, two, NB, Hl, -1)
    view.index_copy_(2, idx, _kv_bytes_pattern(kv, blocks, tp_rank, tp, total_heads, tag))


def _verify(kv, blocks, tp_rank, tp, total_heads, tag) -> bool:
    idx = torch.tensor(blocks, device=kv.device)
    L, two, NB, Hl, BS, D = kv.shape
    got = kv.view(torch.uint8).view(L, two, NB, Hl, -1).index_select(2, idx)
    return bool(torch.equal(got, _kv_bytes_pattern(kv, blocks, tp_rank, tp, total_heads, tag)))


def _wait(pred, what: str, timeout: float = 60.0) -> None:
    t0 = time.time()
    while not pred():
        if time.time() - t0 > timeout:
            raise RuntimeError(f"preflight: {what} did not complete in {timeout}s")
        time.sleep(0.0005)


def kv_check_one_sided(dp, engine_id: str, is_prefill: bool, pre: list[str], dec: list[str], tp_of: dict,
                       barrier, nblocks: int = 3) -> dict:
    """One-sided (ipc) transport: every prefill rank writes a pattern (tagged
    by its engine) into blocks of its own on every decode engine, straight
    through the data plane's remote mapping; after `barrier()` (every rank of
    the world) each decode rank checks every prefill engine's blocks byte
    for byte, and every prefill rank READs them back (one-sided copy out of
    the decode caches into fresh blocks of its own) and checks the round
    trip; a last barrier keeps the decode blocks still until then."""
    t0 = time.perf_counter()
    H = dp.total_kv_heads
    blocks = list(range(1, 1 + nblocks))
    res = {"pairs": 0, "write_ok": 0, "read_ok": 0, "one_sided": True}
    for i, pe in enumerate(pre):
        dst_blocks = list(range(1 + nblocks * (i + 1), 1 + nblocks * (i + 2)))
        for de in dec:
            if engine_id not in (pe, de):
                continue
            res["pairs"] += 1
            if is_prefill:
                rid = f"__preflight_w_{pe}_{de}"
                _fill(dp.kv, blocks, dp.rank, tp_of[pe], H, tag=3 + i)
                dp.begin_send(rid, blocks, de, tp_of[de], dst_block_ids=dst_blocks)
                dp.end_forward()
                _wait(lambda: rid in dp.poll_sends() or rid not in dp.sends, "preflight one-sided WRITE")
    if dp.kv.is_cuda:
        torch.cuda.synchronize(dp.kv.device)
    barrier()
    if not is_prefill:
        for i, pe in enumerate(pre):
            dst_blocks = list(range(1 + nblocks * (i + 1), 1 + nblocks * (i + 2)))
            res["write_ok"] += _verify(dp.kv, dst_blocks, dp.rank, tp_of[engine_id], H, tag=3 + i)
    else:
        i = pre.index(engine_id)
        src_blocks = list(range(1 + nblocks * (i + 1), 1 + nblocks * (i + 2)))
        back = list(range(1 + nblocks, 1 + 2 * nblocks))  # not the pattern's own blocks
        for de in dec:
            rid = f"__preflight_r_{engine_id}_{de}"
            dp.kv.view(torch.uint8)[:, :, back].zero_()
            dp.read_one_sided(rid, back, de, tp_of[de], src_blocks)
            _wait(lambda: rid in dp.reads_landed(), "preflight one-sided READ")
            dp.finish_read(rid)
            dp.poll_reads()
            if dp.kv.is_cuda:
                torch.cuda.synchronize(dp.kv.device)
            res["read_ok"] += _verify(dp.kv, back, dp.rank, tp_of[engine_id], H, tag=3 + i)
    barrier()
    res["ok"] = (res["read_ok"] if is_prefill else res["write_ok"]) == res["pairs"]
    res["ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    return res


def kv_check(dp, engine_id: str, is_prefill: bool, ranks_of: dict, pre: list[str], dec: list[str],
             tp_of: dict, nblocks: int = 3) -> dict:
    """Every rank of the world calls this (ranks outside a pair skip it).
    `dp` is this rank's KVDataPlane; `tp_of[engine]` the engines' TP sizes.
    Uses blocks [1, 1 + nblocks) of every cache (the engines are idle)."""
    t0 = time.perf_counter()
    H = dp.total_kv_heads
    blocks = list(range(1, 1 + nblocks))
    dst_blocks = list(range(1 + nblocks, 1 + 2 * nblocks))  # the receiving side lands them elsewhere
    res = {"pairs": 0, "write_ok": 0, "read_ok": 0}
    for pe in pre:
        for de in dec:
            if engine_id not in (pe, de):
                continue
            rid_w, rid_r = f"__preflight_w_{pe}_{de}", f"__preflight_r_{pe}_{de}"
            ptp, dtp = tp_of[pe], tp_of[de]
            if is_prefill:
                # WRITE: my heads' pattern -> the decode engine
                _fill(dp.kv, blocks, dp.rank, ptp, H, tag=1)
                dp.begin_send(rid_w, blocks, de, dtp)
                dp.end_forward()
                _wait(lambda: rid_w in dp.poll_sends() or rid_w not in dp.sends, "preflight WRITE send")
                # READ: pull the decode engine's pattern (tag 2)
                dp.post_read(rid_r, dst_blocks, de, dtp)
                _wait(lambda: rid_r in dp.reads_landed(), "preflight READ")
                dp.finish_read(rid_r)
                dp.poll_reads()
                if dp.kv.is_cuda:
                    torch.cuda.synchronize(dp.kv.device)
                res["read_ok"] += _verify(dp.kv, dst_blocks, dp.rank, ptp, H, tag=2)
            else:
                dp.post_recv_batch(pe, ptp, [(rid_w, nblocks, dst_blocks)])
                _wait(lambda: rid_w in dp.recvs_landed(), "preflight WRITE receive")
                dp.finish_recv(rid_w)
                dp.poll_recvs()
                if dp.kv.is_cuda:
                    torch.cuda.synchronize(dp.kv.device)
                res["write_ok"] += _verify(dp.kv, dst_blocks, dp.rank, dtp, H, tag=1)
                _fill(dp.kv, blocks, dp.rank, dtp, H, tag=2)
                dp.serve_read(rid_r, blocks, pe, ptp)
                _wait(lambda: dp.poll_served() == 0, "preflight READ serve")
            res["pairs"] += 1
    res["ok"] = res["write_ok" if not is_prefill else "read_ok"] == res["pairs"]
    res["ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    return res
