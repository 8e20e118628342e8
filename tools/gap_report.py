"""Idle gaps inside prefill forwards, from a rocprofv3 kernel-trace CSV of
tools/loopback_disagg.py ("a trace of a loopback prefill
step showing no idle gaps at layer-group boundaries").

A prefill forward is `layers` consecutive `prefill_attn` dispatches (one
per layer; default 32); its window runs from the forward's first to its
last attention kernel.  Per window: GPU busy fraction (union of
all streams' kernels), the largest idle gaps, and how many KV pack/unpack
kernels (`kv_copy`) ran inside it.  The tool's first half of the forwards
runs without any transfer (phase A), the second half streams KV (phase B).

  python tools/gap_report.py trace_kernel_trace.csv [layers]
"""
import csv
import sys


def main(path: str) -> None:
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    attn = [k for k in ks if "prefill_attn" in k[2]]
    layers = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    wins = [attn[i:i + layers] for i in range(0, len(attn) - layers + 1, layers)]  # one forward = one per layer
    print(f"{len(wins)} prefill forwards ({len(attn)} attention dispatches)")
    for i, w in enumerate(wins):
        t0, t1 = w[0][0], w[-1][1]
        inside = [k for k in ks if k[1] > t0 and k[0] < t1]
        busy, ce, gaps = 0, None, []
        cs = None
        for s, e, _ in inside:
            s, e = max(s, t0), min(e, t1)
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                    gaps.append(s - ce)
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        span = t1 - t0
        gaps.sort(reverse=True)
        packs = sum(1 for k in inside if "kv_copy" in k[2])
        print(f"forward {i}: {span / 1e6:7.2f} ms, GPU busy {100 * busy / span:5.1f} %, {len(gaps)} gaps, "
              f"> 20 us: {sum(1 for g in gaps if g > 20e3)}, largest (us): "
              + ", ".join(f"{g / 1e3:.1f}" for g in gaps[:4]) + f"; kv_copy kernels inside: {packs}")


if __name__ == "__main__":
    main(sys.argv[1])
