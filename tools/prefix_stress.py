"""Engine-level stress of prefix-cache-heavy traffic (the router_bench random
mode on one worker): shared-prefix prompts under KV pressure; reports any
engine step slower than --slow-s with its batch composition."""
import argparse, json, os, random, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from dynamo_exp_amd.engine.request import SamplingParams

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3-8b")
ap.add_argument("--blocks", type=int, default=384)
ap.add_argument("--groups", type=int, default=16)
ap.add_argument("--prefix", type=int, default=2048)
ap.add_argument("--suffix", type=int, default=347)
ap.add_argument("--osl", type=int, default=16)
ap.add_argument("--conc", type=int, default=12)
ap.add_argument("--requests", type=int, default=300)
ap.add_argument("--slow-s", type=float, default=0.5)
ap.add_argument("--device", default="cuda")
a = ap.parse_args()
eng = LLMEngine(EngineConfig(model=a.model, device=a.device, block_size=64, max_model_len=4096, num_gpu_blocks=a.blocks,
                             max_num_seqs=64, use_cuda_graph=a.device != "cpu"))
if a.device != "cpu":
    eng.warmup()
rng = random.Random(0)
V = eng.model_cfg.vocab_size
pre = [[rng.randrange(1000, V - 1000) for _ in range(a.prefix)] for _ in range(a.groups)]
st = dict(n=0, done=0)
def submit():
    st["n"] += 1
    p = rng.choice(pre) + [rng.randrange(1000, V - 1000) for _ in range(a.suffix)]
    def cb(req, toks, lps, fin):
        if fin:
            st["done"] += 1
            if st["n"] < a.requests:
                submit()
    eng.add_request(f"r{st['n']}", p, SamplingParams(max_tokens=a.osl, min_tokens=a.osl, ignore_eos=True), on_output=cb)
for _ in range(a.conc):
    submit()
slow = []
t_all = time.perf_counter()
steps = 0
while eng.has_unfinished():
    sched = eng.scheduler
    t0 = time.perf_counter()
    eng.step()
    torch.cuda.synchronize() if a.device != "cpu" else None
    dt = time.perf_counter() - t0
    steps += 1
    b = eng.last_batch
    if dt > a.slow_s and b is not None:
        info = {"step": steps, "s": round(dt, 3), "kind": b.kind,
                "rows": [(len(r.prompt), r.num_computed, n) for r, n in zip(b.requests, b.num_new or [])][:40]}
        slow.append(info)
        print("SLOW", json.dumps(info), flush=True)
print(json.dumps({"steps": steps, "wall_s": round(time.perf_counter() - t_all, 2), "done": st["done"],
                  "slow_steps": len(slow), "preemptions": eng.scheduler.preemptions}), flush=True)
