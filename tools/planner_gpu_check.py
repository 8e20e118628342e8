#!/usr/bin/env python3
"""The planner actuating REAL HIP engines on one MI355X (the planner had only ever scaled
simulated workers).

`dynamo serve graphs.disagg_router:Frontend` with Llama-3-8B engines (random-init weights), starting at one
decode and one prefill worker that share the GPU (`resources.gpu` fractions, host-staged KV transfer), the local
planner in operating mode (`--policy utilization` or `rate`, 5 s adjustment interval, a budget of 3 workers).  A
closed loop of streaming completions whose prompts all prefill remotely overloads the single prefill worker; the planner must add
a prefill worker (the supervisor starts a new engine process on the GPU, it registers, pulls the shared prefill
queue), and after the load stops remove one again (lease revoked: graceful drain).  Checks: an `add
PrefillWorker` action, a second prefill instance whose `mock` endpoint reports dequeued prompts (it served), a
later `remove PrefillWorker`, and every request completing.  Both workers share one device, so this proves the
actuation path, not a capacity gain (the capacity study is tools/planner_bench.py on the timing model).

    python tools/planner_gpu_check.py --out profiles/r5_planner_real_engines.json
    python tools/planner_gpu_check.py --policy rate --out profiles/r5_planner_real_engines_rate.json
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def log(msg: str) -> None:
    print(f"[planner_gpu_check] {msg}", flush=True)


async def prefill_instances(cp: str) -> dict:
    """{instance id: mock reply} of every registered PrefillWorker."""
    from dynamo_exp_amd.runtime.distributed import DistributedRuntime

    drt = await DistributedRuntime.create(cp, is_static=True)
    try:
        client = await drt.namespace("dynamo").component("PrefillWorker").endpoint("mock").client()
        await asyncio.sleep(1.0)
        out = {}
        for iid in client.instance_ids():
            try:
                async def first():
                    async for r in await client.direct({}, iid):
                        return r
                out[str(iid)] = await asyncio.wait_for(first(), 5)
            except Exception as e:  # noqa: BLE001
                out[str(iid)] = {"error": repr(e)}
        return out
    finally:
        await drt.close(1)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--load-s", type=float, default=45.0)
    ap.add_argument("--concurrency", type=int, default=48)
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--gpu-share", default="0.25", help="resources.gpu of each worker (0: CPU engines, a dry run)")
    ap.add_argument("--policy", default="utilization", choices=["utilization", "rate"])
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    import httpx

    work = tempfile.mkdtemp(prefix="dx_planner_gpu_")
    cp_port, http_port = _free(), _free()
    cp = f"127.0.0.1:{cp_port}"
    plog_dir = os.path.join(work, "planner")
    env = dict(os.environ, PYTHONPATH=ROOT, DYN_STATE_DIR=work, DYN_LOG="warning", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "dynamo_exp_amd.sdk.serve", "graphs.disagg_router:Frontend",
           "-f", "configs/disagg_router.yaml", f"--Frontend.port={http_port}", f"--Frontend.served_model_name={a.model}",
           f"--Common.model={a.model}", "--Common.block-size=64", "--Common.max-model-len=4096",
           "--Worker.ServiceArgs.workers=1", f"--Worker.ServiceArgs.resources.gpu={a.gpu_share}",
           "--PrefillWorker.ServiceArgs.workers=1", f"--PrefillWorker.ServiceArgs.resources.gpu={a.gpu_share}",
           "--Worker.num-gpu-blocks=4096", "--Worker.max-num-seqs=64", "--PrefillWorker.num-gpu-blocks=1024",
           "--Worker.kv-transport=host", "--PrefillWorker.kv-transport=host",
           "--Worker.max-local-prefill-length=64", "--Worker.max-prefill-queue-size=1000",
           "--enable-local-planner", "--Planner.no-operation=false", f"--Planner.policy={a.policy}",
           "--Planner.adjustment-interval=5", "--Planner.metric-pulling-interval=1", "--Planner.max-gpu-budget=3",
           f"--Planner.log-dir={plog_dir}", "--control-plane", cp]
    serve_log = os.path.join(work, "serve.log")
    proc = subprocess.Popen(cmd, cwd=os.path.join(ROOT, "examples", "llm"), env=env, start_new_session=True,
                            stdout=open(serve_log, "w"), stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{http_port}"
    res: dict = {"config": {"model": a.model, "start": f"1P1D on one GPU ({a.gpu_share} each)", "policy": a.policy,
                            "adjustment_interval_s": 5, "max_gpu_budget": 3, "load_s": a.load_s,
                            "concurrency": a.concurrency, "isl_chars": a.isl}}
    rc = 1
    try:
        t0 = time.time()
        while True:
            if proc.poll() is not None:
                raise RuntimeError(f"serve exited early (see {serve_log})")
            try:
                r = httpx.post(f"{url}/v1/completions", timeout=60, json={
                    "model": a.model, "prompt": "warm up " * 200, "max_tokens": 4, "nvext": {"ignore_eos": True}})
                if r.status_code == 200 and "choices" in r.json():
                    break
            except Exception:  # noqa: BLE001 -- still starting
                pass
            if time.time() - t0 > 600:
                raise RuntimeError("graph not ready after 600 s")
            time.sleep(2.0)
        log(f"graph ready in {time.time() - t0:.0f} s; closed-loop load for {a.load_s:.0f} s")
        res["ready_s"] = round(time.time() - t0, 1)
        t_load = time.time()
        lg = subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "loadgen.py"), "--url", url, "--model", a.model,
                               "--isl", str(a.isl), "--osl", "16", "--isl-unit", "chars", "--concurrency",
                               str(a.concurrency), "--requests-per-conc", str(max(4, int(a.load_s * 30 / a.concurrency))),
                               "--warmup-per-conc", "0", "--client", "raw",
                               "--out", os.path.join(work, "load.json")],
                              stdout=open(os.path.join(work, "loadgen.out"), "w"), stderr=subprocess.STDOUT)
        # sample the prefill pool mid-load too: a policy may shrink it again before the load ends
        res["instances_mid_load"] = {}
        while lg.poll() is None and time.time() - t_load < a.load_s + 600:
            if time.time() - t_load > 0.75 * a.load_s and not res["instances_mid_load"]:
                res["instances_mid_load"] = asyncio.run(prefill_instances(cp))
            time.sleep(1.0)
        lg.wait(60)
        res["load_wall_s"] = round(time.time() - t_load, 1)
        with open(os.path.join(work, "loadgen.out")) as f:
            res["loadgen_tail"] = f.read().strip().splitlines()[-1:]
        res["instances_after_load"] = asyncio.run(prefill_instances(cp))
        log(f"prefill instances after the load: {res['instances_after_load']}")
        time.sleep(40)  # quiet period: the planner should remove a prefill worker
        res["instances_after_quiet"] = asyncio.run(prefill_instances(cp))
        acts = []
        with open(os.path.join(plog_dir, "planner.jsonl")) as f:
            for line in f:
                e = json.loads(line)
                if e.get("kind") == "adjust" and e.get("actions"):
                    acts.append({"t": round(e["t"], 1), "actions": e["actions"], "n_prefill": e.get("n_prefill"),
                                 "n_decode": e.get("n_decode")})
        res["planner_actions"] = acts
        added = any(["add", "PrefillWorker"] in x["actions"] or ("add", "PrefillWorker") in x["actions"]
                    for x in acts)
        removed = any(["remove", "PrefillWorker"] in x["actions"] or ("remove", "PrefillWorker") in x["actions"]
                      for x in acts)
        # a prefill remove within 30 s of a prefill add is a flap (the rate policy's scale-down delay forbids it)
        adds = [x["t"] for x in acts if ["add", "PrefillWorker"] in x["actions"] or ("add", "PrefillWorker") in x["actions"]]
        flaps = sum(1 for x in acts if (["remove", "PrefillWorker"] in x["actions"]
                                        or ("remove", "PrefillWorker") in x["actions"])
                    and any(0 <= x["t"] - t < 30 for t in adds))
        served = [max((snap.get(i) or {}).get("dequeued", 0) if isinstance(snap.get(i), dict) else 0
                      for snap in (res["instances_mid_load"], res["instances_after_load"]))
                  for i in set(res["instances_mid_load"]) | set(res["instances_after_load"])]
        res["checks"] = {"added_prefill_worker": added,
                         "prefill_instances_after_load": len(res["instances_after_load"]),
                         "instances_that_served": sum(1 for d in served if d and d > 0),
                         "removed_prefill_worker": removed, "prefill_flaps": flaps,
                         "prefill_instances_after_quiet": len(res["instances_after_quiet"])}
        ok = added and removed and res["checks"]["instances_that_served"] >= 2 and (a.policy != "rate" or flaps == 0)
        res["ok"] = ok
        rc = 0 if ok else 1
    except Exception as e:  # noqa: BLE001
        res["error"] = repr(e)
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(90)
        except Exception:  # noqa: BLE001
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except Exception:  # noqa: BLE001
                pass
        with open(serve_log) as f:
            res["serve_log_tail"] = f.read().splitlines()[-15:]
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        log(json.dumps({k: res.get(k) for k in ("ok", "checks", "error")}))
    return rc


if __name__ == "__main__":
    sys.exit(main())
