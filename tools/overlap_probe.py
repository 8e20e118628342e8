"""Does decode attention overlap prefill attention when launched on a side
stream (models/llama.py overlap_decode_attn)?  Times, at mixed-step shapes,
each kernel alone, both back to back on one stream, and both forked onto two
streams (prefill first on the main stream, decode on the side stream; and the
reverse order).

  python -m tools.overlap_probe
"""
import math

import torch

from dynamo_exp_amd import ops


def timed(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    Hq, Hkv, D, bs = 32, 8, 128, 64
    sc = 1 / math.sqrt(D)
    # prefill: 2 prompts x 2800 new tokens (a mixed step's ~5600 prompt tokens)
    L, nseq = 2800, 2
    nb = nseq * (L // bs + 1) + 4
    kp = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vp = torch.randn_like(kp)
    btp = torch.arange(nb - 4, dtype=torch.int32, device="cuda").view(nseq, -1)
    qp = torch.randn(nseq * L, Hq, D, device="cuda", dtype=torch.bfloat16)
    cu = torch.arange(0, nseq * L + 1, L, dtype=torch.int32, device="cuda")
    ctxp = torch.full((nseq,), L, dtype=torch.int32, device="cuda")
    work = torch.tensor(ops.prefill_work_list([L] * nseq, [L] * nseq, Hq, Hkv), dtype=torch.int32, device="cuda")
    op = torch.empty_like(qp)
    # decode: 120 streams at ~3100 context
    B, Ld = 120, 3100
    nbps = Ld // bs + 1
    kd = torch.randn(B * nbps, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vd = torch.randn_like(kd)
    btd = torch.randperm(B * nbps, device="cuda").to(torch.int32).view(B, nbps)
    qd = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    ctxd = torch.randint(Ld - 150, Ld, (B,), dtype=torch.int32, device="cuda")
    od = torch.empty_like(qd)
    mp = ops.decode_num_parts(B, Hkv, Ld)
    ws = ops.decode_workspace(B, Hq, D, mp, "cuda")
    side = torch.cuda.Stream()

    def pre():
        ops.prefill_attention(qp, kp, vp, btp, cu, ctxp, sc, op, work=work)

    def dec():
        ops.decode_attention(qd, kd, vd, btd, ctxd, sc, od, mp, workspace=ws)

    def forked(first_prefill=True):
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        if first_prefill:
            pre()
        with torch.cuda.stream(side):
            dec()
        if not first_prefill:
            pre()
        main.wait_stream(side)

    for rnd in range(3):
        r = {"prefill": timed(pre), "decode": timed(dec), "serial": timed(lambda: (pre(), dec())),
             "fork_p_first": timed(lambda: forked(True)), "fork_d_first": timed(lambda: forked(False))}
        print(rnd, {k: round(v, 1) for k, v in r.items()}, flush=True)


if __name__ == "__main__":
    main()
