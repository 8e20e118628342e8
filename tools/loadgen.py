"""genai-perf-style load generator for the OpenAI frontend (reference
examples/llm/benchmarks/perf.sh:17-54 and the planner's sinusoidal trace,
docs/guides/planner_benchmark/sin_synth.py).

Concurrency sweep (closed loop, `--requests-per-conc` x concurrency requests
after `--warmup-per-conc` x concurrency warm-up requests):
    python tools/loadgen.py --url http://127.0.0.1:8000 --model llama3-8b --isl 3000 --osl 150 \
        --concurrency 1,8,32,128 --out sweep.json
Open-loop sinusoidal request rate (rate(t) = mid + amp*sin(2*pi*t/period)):
    python tools/loadgen.py --trace sin --min-rate 5 --max-rate 20 --period 150 --duration 600 ...

Requests are streaming chat completions with `ignore_eos` and
`min_tokens = max_tokens = osl` (fixed output length, as the reference's
methodology) and synthetic prompts of ~ISL tokens.  Reports output tok/s,
tok/s/user, TTFT / ITL / latency p50 and p99 per point.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import math
import random
import time

import httpx

WORDS = ("alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu nu xi omicron pi rho sigma tau "
         "upsilon phi chi psi omega").split()


ISL_UNIT = {"unit": "words"}


def make_prompt(rng: random.Random, isl: int) -> str:
    """~isl tokens: one short word per token for BPE tokenizers (`words`), or
    isl characters for byte-level tokenizers (`chars`, e.g. the synthetic
    tokenizer of random-init presets)."""
    if ISL_UNIT["unit"] == "chars":
        return "".join(rng.choices("abcdefghijklmnopqrstuvwxyz ", k=isl))
    return " ".join(rng.choices(WORDS, k=isl))


class PromptSource:
    """Synthetic prompts of ~isl tokens.  With prefix groups, every prompt is
    one of `groups` shared prefixes of `prefix_len` tokens (e.g. a system prompt
    or a conversation history, chosen uniformly) followed by a unique suffix --
    the shape that makes KV-aware routing pay off."""

    def __init__(self, rng: random.Random, isl: int, groups: int = 0, prefix_len: int = 0):
        self.rng, self.isl = rng, isl
        self.prefixes = [make_prompt(rng, prefix_len) for _ in range(groups)] if groups and prefix_len else []

    def __call__(self) -> str:
        if not self.prefixes:
            return make_prompt(self.rng, self.isl)
        pre = self.rng.choice(self.prefixes)
        n = max(1, self.isl - len(pre.split()) if ISL_UNIT["unit"] == "words" else self.isl - len(pre))
        sep = " " if ISL_UNIT["unit"] == "words" else ""
        return pre + sep + make_prompt(self.rng, n)


def pct(xs: list[float], p: float) -> float | None:
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(len(xs) * p))]


async def one_request(client: httpx.AsyncClient, url: str, model: str, prompt: str, osl: int) -> dict:
    # osl = output tokens (max_tokens = min_tokens)
    body = {"model": model, "messages": [{"role": "user", "content": prompt}], "stream": True,
            "max_tokens": osl, "min_tokens": osl, "nvext": {"ignore_eos": True},
            "stream_options": {"include_usage": True}}
    t0 = time.perf_counter()
    first = last = None
    chunks = 0
    usage = None
    gaps = []
    times = []
    async with client.stream("POST", f"{url}/v1/chat/completions", json=body) as r:
        if r.status_code != 200:
            return {"ok": False, "status": r.status_code}
        async for line in r.aiter_lines():
            if not line.startswith("data: "):
                continue
            data = line[6:]
            if data == "[DONE]":
                break
            ch = json.loads(data)
            if ch.get("usage"):
                usage = ch["usage"]
            if any((c.get("delta") or {}).get("content") for c in ch.get("choices", [])):
                now = time.perf_counter()
                if first is None:
                    first = now
                else:
                    gaps.append(now - last)
                last = now
                times.append(now)
                chunks += 1
    end = time.perf_counter()
    out_tokens = usage["completion_tokens"] if usage else chunks
    return {"ok": True, "ttft": (first - t0) if first else None, "latency": end - t0, "out_tokens": out_tokens,
            "itl": (sum(gaps) / len(gaps)) if gaps else None, "t_end": end, "times": times}


class RawPool:
    """Keep-alive HTTP/1.1 connections over bare asyncio streams, SSE parsed
    by hand (`--client raw`): httpx costs tens of microseconds of client CPU
    per streamed chunk, which at tens of requests/s x 150 tokens makes the
    load generator, not the server, fall behind an open-loop schedule when
    both share a small host."""

    def __init__(self, url: str):
        host, port = url.split("//", 1)[1].rstrip("/").rsplit(":", 1)
        self.host, self.port = host, int(port)
        self.free: list = []

    IDLE_S = 10.0  # well under the server's keep-alive timeout (30 s)

    async def get(self, fresh: bool = False):
        now = time.monotonic()
        while self.free and not fresh:
            r, w, t = self.free.pop()
            if not w.is_closing() and not r.at_eof() and now - t < self.IDLE_S:
                return r, w
            w.close()
        return await asyncio.open_connection(self.host, self.port, limit=1 << 20)

    def put(self, conn) -> None:
        self.free.append((conn[0], conn[1], time.monotonic()))

    async def close(self) -> None:
        for _, w, _ in self.free:
            w.close()
        self.free.clear()


async def one_request_raw(pool: RawPool, model: str, prompt: str, osl: int) -> dict:
    body = json.dumps({"model": model, "messages": [{"role": "user", "content": prompt}], "stream": True,
                       "max_tokens": osl, "min_tokens": osl, "nvext": {"ignore_eos": True},
                       "stream_options": {"include_usage": True}}).encode()
    req = (b"POST /v1/chat/completions HTTP/1.1\r\nhost: x\r\ncontent-type: application/json\r\n"
           b"content-length: %d\r\n\r\n%b" % (len(body), body))
    t0 = time.perf_counter()
    first = last = None
    chunks = 0
    usage = None
    gaps = []
    times = []
    r, w = await pool.get()
    try:
        w.write(req)
        try:
            head = await r.readuntil(b"\r\n\r\n")
        except (OSError, asyncio.IncompleteReadError):
            # a pooled keep-alive connection the server closed meanwhile: one
            # retry on a fresh connection (nothing of the response was read)
            w.close()
            r, w = await pool.get(fresh=True)
            w.write(req)
            head = await r.readuntil(b"\r\n\r\n")
        if not head.startswith(b"HTTP/1.1 200"):
            w.close()
            return {"ok": False, "status": head[:40].decode(errors="replace")}
        buf = b""
        while True:
            size = int((await r.readuntil(b"\r\n"))[:-2], 16)
            data = await r.readexactly(size + 2)
            if size == 0:
                break
            buf += data[:-2]
            while (k := buf.find(b"\n\n")) >= 0:
                ev, buf = buf[:k], buf[k + 2:]
                if not ev.startswith(b"data: {"):
                    continue
                if b'"usage"' in ev:
                    usage = json.loads(ev[6:]).get("usage") or usage
                if b'"content"' in ev and b'"content": ""' not in ev:
                    now = time.perf_counter()
                    if first is None:
                        first = now
                    else:
                        gaps.append(now - last)
                    last = now
                    times.append(now)
                    chunks += 1
    except (OSError, asyncio.IncompleteReadError, ValueError) as e:
        w.close()
        return {"ok": False, "error": repr(e)}
    pool.put((r, w))
    end = time.perf_counter()
    out_tokens = usage["completion_tokens"] if usage else chunks
    return {"ok": True, "ttft": (first - t0) if first else None, "latency": end - t0, "out_tokens": out_tokens,
            "itl": (sum(gaps) / len(gaps)) if gaps else None, "t_end": end, "times": times}


def summarize(results: list[dict], wall: float, conc: int | None, window: tuple | None = None) -> dict:
    """window = (t_a, t_b): also the steady-state rate -- streamed tokens
    that arrived inside the window / its length (closed loop: from the start
    of the measured round to the moment the first stream ran out of requests,
    i.e. while all `conc` streams were in flight, the bench's regime)."""
    ok = [r for r in results if r.get("ok")]
    toks = sum(r["out_tokens"] for r in ok)
    s = {"requests": len(results), "ok": len(ok), "wall_s": round(wall, 3),
         "output_tok_s": round(toks / wall, 2) if wall > 0 else 0.0, "req_s": round(len(ok) / wall, 3) if wall else 0}
    for name in ("ttft", "itl", "latency"):
        xs = [r[name] for r in ok if r.get(name) is not None]
        s[f"{name}_p50_ms"] = round(pct(xs, 0.5) * 1000, 2) if xs else None
        s[f"{name}_p99_ms"] = round(pct(xs, 0.99) * 1000, 2) if xs else None
        s[f"{name}_mean_ms"] = round(sum(xs) / len(xs) * 1000, 2) if xs else None
        s[f"{name}_max_ms"] = round(max(xs) * 1000, 2) if xs else None
    s["ttft_over_1s"] = sum(1 for r in ok if (r.get("ttft") or 0) > 1.0)
    errs: dict = {}
    for r in results:
        if not r.get("ok"):
            key = str(r.get("status") or r.get("error") or "unknown")[:80]
            errs[key] = errs.get(key, 0) + 1
    if errs:
        s["errors"] = errs
    if conc:
        s["concurrency"] = conc
        s["tok_s_per_user"] = round(s["output_tok_s"] / conc, 2)
    if window and window[1] > window[0]:
        n = sum(1 for r in ok for t in r.get("times", ()) if window[0] <= t < window[1])
        s["steady_window_s"] = round(window[1] - window[0], 3)
        s["steady_output_tok_s"] = round(n / (window[1] - window[0]), 2)
    return s


async def closed_loop(a, conc: int, rng: random.Random) -> dict:
    src = PromptSource(rng, a.isl, getattr(a, "prefix_groups", 0), getattr(a, "prefix_len", 0))
    raw = getattr(a, "client", "httpx") == "raw"
    pool = RawPool(a.url) if raw else None
    c = None if raw else httpx.AsyncClient(timeout=httpx.Timeout(a.timeout),
                                          limits=httpx.Limits(max_connections=conc + 8))
    try:
        async def one(osl: int):
            if raw:
                return await one_request_raw(pool, a.model, src(), osl)
            return await one_request(c, a.url, a.model, src(), osl)

        async def worker(i: int, warm: list, sink: list) -> tuple[float, float]:
            """Warm-up requests, then measured ones, back to back (no barrier
            between the phases: a lock-step restart of every stream would put
            a prefill burst in the measured round).  The first warm-up request
            of stream i is cut to (i + 1) / conc of the OSL (bench.py's
            stagger), so the streams finish -- and re-admit -- spread over one
            OSL instead of in waves."""
            for k in range(a.warmup_per_conc):
                osl = max(1, (i + 1) * a.osl // conc) if k == 0 and a.stagger else a.osl
                warm.append(await one(osl))
            t_w = time.perf_counter()
            for _ in range(a.requests_per_conc):
                sink.append(await one(a.osl))
            return t_w, time.perf_counter()

        warm: list = []
        res: list = []
        t0 = time.perf_counter()
        marks = await asyncio.gather(*(worker(i, warm, res) for i in range(conc)))
        # steady state: every stream past its warm-up, none out of requests yet;
        # tokens of any request that arrived inside that window count
        t_a, t_b = max(m[0] for m in marks), min(m[1] for m in marks)
        t_meas = min((r["t_end"] - r["latency"] for r in res if r.get("ok")), default=t0)
        s = summarize(res, time.perf_counter() - t_meas, conc)
        if t_b > t_a:
            n = sum(1 for r in warm + res if r.get("ok") for t in r.get("times", ()) if t_a <= t < t_b)
            s["steady_window_s"] = round(t_b - t_a, 3)
            s["steady_output_tok_s"] = round(n / (t_b - t_a), 2)
        return s
    finally:
        if pool is not None:
            await pool.close()
        if c is not None:
            await c.aclose()


async def sin_trace(a, rng: random.Random) -> dict:
    """Open loop: Poisson arrivals at rate(t) = mid + amp * sin(2 pi t / period).
    Arrival times are drawn up front and kept on an absolute schedule, so a
    busy client cannot silently thin the trace; `schedule_lag_p99_ms` reports
    how late requests actually went out."""
    mid, amp = (a.max_rate + a.min_rate) / 2, (a.max_rate - a.min_rate) / 2
    arrivals, t = [], 0.0
    while True:  # thinning-free: exponential gaps at the rate at the current time
        t += rng.expovariate(max(0.1, mid + amp * math.sin(2 * math.pi * t / a.period)))
        if t >= a.duration:
            break
        arrivals.append(t)
    res: list = []
    lags: list = []
    src = PromptSource(rng, a.isl, getattr(a, "prefix_groups", 0), getattr(a, "prefix_len", 0))
    raw = getattr(a, "client", "httpx") == "raw"
    pool = RawPool(a.url) if raw else None
    c = None if raw else httpx.AsyncClient(timeout=httpx.Timeout(a.timeout),
                                          limits=httpx.Limits(max_connections=4096))
    try:
        tasks = []
        t0 = time.perf_counter()
        for at in arrivals:
            delay = t0 + at - time.perf_counter()
            if delay > 0:
                await asyncio.sleep(delay)
            lags.append(max(0.0, time.perf_counter() - t0 - at))
            prompt = src()  # shared-prefix groups too (--prefix-groups), as in the closed loop

            async def go(prompt=prompt):
                if raw:
                    res.append(await one_request_raw(pool, a.model, prompt, a.osl))
                else:
                    res.append(await one_request(c, a.url, a.model, prompt, a.osl))

            tasks.append(asyncio.create_task(go()))
        await asyncio.gather(*tasks)
        out = summarize(res, time.perf_counter() - t0, None)
        out["scheduled"] = len(arrivals)
        out["schedule_lag_p99_ms"] = round(pct(lags, 0.99) * 1000, 2) if lags else None
        return out
    finally:
        if pool is not None:
            await pool.close()
        if c is not None:
            await c.aclose()


def main(argv=None):
    ap = argparse.ArgumentParser(prog="loadgen")
    ap.add_argument("--url", default="http://127.0.0.1:8000")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--isl", type=int, default=3000)
    ap.add_argument("--osl", type=int, default=150)
    ap.add_argument("--concurrency", default="1,2,4,8,16,32,64,128,256")
    ap.add_argument("--requests-per-conc", type=int, default=10)
    ap.add_argument("--warmup-per-conc", type=int, default=2)
    ap.add_argument("--trace", choices=["closed", "sin"], default="closed")
    ap.add_argument("--min-rate", type=float, default=5.0)
    ap.add_argument("--max-rate", type=float, default=20.0)
    ap.add_argument("--period", type=float, default=150.0)
    ap.add_argument("--duration", type=float, default=600.0)
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--isl-unit", choices=["words", "chars"], default="words")
    ap.add_argument("--stagger", type=int, default=1,
                    help="closed loop: stream i's first warm-up request generates (i + 1) / C of the OSL (1 = on)")
    ap.add_argument("--client", choices=["httpx", "raw"], default="httpx",
                    help="raw: bare asyncio HTTP/1.1 client (open-loop traces at high request rates)")
    ap.add_argument("--prefix-groups", type=int, default=0, help="shared-prefix groups (0 = all prompts distinct)")
    ap.add_argument("--prefix-len", type=int, default=0, help="tokens of each group's shared prefix")
    a = ap.parse_args(argv)
    ISL_UNIT["unit"] = a.isl_unit
    rng = random.Random(a.seed)
    if a.trace == "sin":
        results = [asyncio.run(sin_trace(a, rng))]
    else:
        results = [asyncio.run(closed_loop(a, int(c), rng)) for c in a.concurrency.split(",")]
    for r in results:
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"isl": a.isl, "osl": a.osl, "model": a.model, "points": results}, f, indent=1)
    return results


if __name__ == "__main__":
    main()
