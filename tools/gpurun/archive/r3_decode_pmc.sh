#!/bin/bash
# PMC pass over decode attention, bf16 vs fp8 KV (one counter set, kernel trace only)
set -o pipefail
mkdir -p gpurun_out/dpmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/dpmc -o dpmc --output-format csv -- python3 -m tools.decode_pmc_driver > gpurun_out/dpmc/run.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/dpmc/run.log; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/dpmc | head -12
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob("gpurun_out/dpmc/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r.get("Kernel_Name", "?")
        if "decode_attn" not in k: continue
        tag = "fp8" if "Lb1ELb1E" in k or "true, true" in k else "bf16"
        rows[tag][r["Counter_Name"]] += float(r["Counter_Value"])
for t, c in rows.items():
    wc = c["SQ_WAVE_CYCLES"] or 1
    print(t, {n: round(v / wc, 3) for n, v in c.items() if n != "SQ_WAVE_CYCLES"}, "VALU insts/VMEM rd", round(c["SQ_INSTS_VALU"] / max(1, c["SQ_INSTS_VMEM_RD"]), 1))
PY
