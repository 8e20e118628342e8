"""Per decode batch size and Llama-3-8B projection: the best config of each
small-M GEMM family (skinny / dstream; round 4 also timed the removed wstream) next to hipBLASLt, timed
over all 32 layers' weights (partials left to the consumer where the
engine does so).  python tools/gemm_family_probe.py"""
import json, sys, torch
sys.path.insert(0, ".")
from dynamo_exp_amd import ops
from dynamo_exp_amd.models.config import get_config
from dynamo_exp_amd.models.llama import LlamaForCausalLM

def timed(fn, reps=2):
    fn(); e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize(); return e0.elapsed_time(e1) * 1e3 / reps

m = LlamaForCausalLM(get_config("llama3-8b"), device=torch.device("cuda:0")).random_init(1)
for M in (16, 32, 48, 64, 80, 96, 112):
    for n in ("qkv", "o", "gate_up", "down"):
        ws = [L[n] for L in m.layers]
        N, K = ws[0].shape
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        row = {"M": M, "proj": n, "lib": round(timed(lambda: [torch.matmul(x, w.t()) for w in ws]) / len(ws), 2)}
        for fam, cfgs in (("skinny", ops.skinny_configs(M, N, K)),
                          ("dstream", ops.dstream_tune_configs(M, N, K))):
            best = None
            for cfg in cfgs:
                if fam == "skinny" and ((M <= 32 and cfg[1] == 64) or (cfg[0] == 128 and M <= 32)):
                    continue
                t = timed(lambda: [ops.skinny_linear(x, w, cfg, partial=n != "gate_up") for w in ws]) / len(ws)
                best = t if best is None or t < best else best
            row[fam] = round(best, 2) if best is not None else None
        print(json.dumps(row), flush=True)
