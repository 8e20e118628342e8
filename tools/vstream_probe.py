"""Bandwidth probes of the register-streamed decode GEMM (csrc/kernels/vstream_gemm.hip)
at M 128: full kernel vs no MFMA vs weights only (fragment-shaped 16 rows x 64 B
loads) vs weights only with lane-linear 8 rows x 128 B loads (probe modes give
wrong results); weights cold over 32 copies.

  python -m tools.vstream_probe
"""
import torch

from dynamo_exp_amd import ops
from dynamo_exp_amd.ops import _k, _skinny_ws, _stream
from tools.skinny_bench import SHAPES, timed


def probe(x, w, out, r, splits, mode):
    M, K = x.shape
    N = w.shape[0]
    st = _stream()
    slabs, tickets = _skinny_ws(x.device, st)
    _k().vstream_probe(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), slabs.data_ptr(),
                       tickets.data_ptr(), M, N, K, r, splits, mode, st)


def main():
    M = 128
    for name, splits in (("gate_up", 1), ("qkv", 2), ("o", 4), ("down", 4)):
        N, K = SHAPES[name]
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(32)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        gb = N * K * 2 / 1e9
        row = {"hipblaslt": timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / 32}
        for r, nw in ((2, 4), (1, 8)):
            cfg = (ops.VSTREAM, 128, r, nw, 4, splits, 0)
            row[f"r{r}w{nw}_full"] = timed(lambda: [ops.skinny_linear(x, w, cfg, out=out) for w in ws]) / 32
            for mode, tag in ((1, "no_mfma"), (2, "w_only"), (3, "w_only_linear")):
                row[f"r{r}w{nw}_{tag}"] = timed(lambda: [probe(x, w, out, r, splits, mode) for w in ws]) / 32
        print(name, M, "splits", splits, {k: f"{v:.1f}us {gb / v * 1e3:.2f}TB/s" for k, v in row.items()}, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
