"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches) and
derive MFMA busy %, LDS bank-conflict rate, wait shares and HBM bytes/s."""
import csv
import glob
import sys
from collections import defaultdict


def load(paths):
    agg = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(float)
    calls = defaultdict(int)
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name") or row.get("Kernel-Name") or "?"
                k = k.replace("(anonymous namespace)::", "").replace("void ", "")
                k = k.split("(")[0][:70]
                c = row.get("Counter_Name")
                v = float(row.get("Counter_Value") or 0)
                if c:
                    agg[k][c] += v
                s, e = row.get("Start_Timestamp"), row.get("End_Timestamp")
                if s and e and c:
                    agg[k]["__dur_" + c] += (int(e) - int(s))
    return agg


def main():
    rows = load(sorted(glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True)))
    for k, c in sorted(rows.items(), key=lambda kv: -max([v for n, v in kv[1].items() if n.startswith("__dur")] or [0])):
        d = {n: v for n, v in c.items() if not n.startswith("__")}
        durs = [v for n, v in c.items() if n.startswith("__dur")]
        t_ns = max(durs) if durs else 0
        out = [f"{k}"]
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            wc = d["SQ_WAVE_CYCLES"]
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in d:
                    out.append(f"{n[3:]}={d[n] / wc:.1%}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d and d["GRBM_GUI_ACTIVE"]:
            out.append(f"MFMA_busy~{d['SQ_VALU_MFMA_BUSY_CYCLES'] / (d['GRBM_GUI_ACTIVE'] / 8 * 256 * 4):.1%}")
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_LDS_IDX_ACTIVE" in d and d["SQ_LDS_IDX_ACTIVE"]:
            out.append(f"LDS_conflict={d['SQ_LDS_BANK_CONFLICT'] / d['SQ_LDS_IDX_ACTIVE']:.1%}")
        if "FETCH_SIZE" in d and t_ns:
            out.append(f"HBM_fetch={d['FETCH_SIZE'] * 1024 / t_ns:.2f}GB/s-ish(KB*1024/ns)")
        out.append("raw=" + ", ".join(f"{n}={v:.3g}" for n, v in sorted(d.items())))
        print(" | ".join(out))


if __name__ == "__main__":
    main()
