#!/bin/bash
# Round 6: PMC passes (one counter set per run, kernel trace only) over the folded-norm kernels at T = 8192.
set -o pipefail
out=${1:-gpurun_out/r6_fold_pmc}
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $out/p1 -o p1 --output-format csv -- python3 tools/fold_pmc_driver.py > $out/p1.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $out/p2 -o p2 --output-format csv -- python3 tools/fold_pmc_driver.py > $out/p2.log 2>&1
rc=$?; echo "pass2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/t -o t --output-format csv -- python3 tools/fold_pmc_driver.py > $out/t.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $out/p1 > $out/summary.txt
python3 tools/pmc_summary.py $out/p2 >> $out/summary.txt
f=$(find $out/t -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $out/kernel_stats.csv
find $out/t -name "*kernel_trace.csv" -delete
cut -c1-300 $out/summary.txt | head -40
