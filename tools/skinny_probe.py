"""Small-M (decode) GEMM probe: hipBLASLt x @ W^T vs the transposed problem
W @ x^T (the weight's N becomes the GEMM's M)."""
import torch, json
from microbench import bench
H, F = 4096, 14336
res = {}
for M in (64, 128, 256):
    for name, (K, N) in {"qkv": (H, 6144), "o": (H, H), "gate_up": (H, 2 * F), "down": (F, H)}.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        a = bench(lambda: torch.matmul(x, w.t()), 50)
        b = bench(lambda: torch.matmul(w, x.t()), 50)
        c = bench(lambda: torch.matmul(w, x.t()).t().contiguous(), 50)
        wt = w.t().contiguous()
        d = bench(lambda: torch.matmul(x, wt), 50)
        gb = N * K * 2 / 1e9
        res[f"{name}_M{M}"] = {"xWt_us": round(a, 1), "Wxt_us": round(b, 1), "Wxt_T_us": round(c, 1),
                               "x_Wkn_us": round(d, 1), "weight_TBs_best": round(gb / min(a, b, c, d) * 1e3, 2)}
        print(name, M, res[f"{name}_M{M}"], flush=True)
