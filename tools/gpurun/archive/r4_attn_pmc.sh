#!/bin/bash
# PMC passes over prefill attention (round-3 loop vs current), one counter set per run, kernel trace only
set -o pipefail
out=${1:-gpurun_out/apmc}
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $out/p1 -o p1 --output-format csv -- python3 -m tools.attn_pmc_driver > $out/p1.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $out/p2 -o p2 --output-format csv -- python3 -m tools.attn_pmc_driver > $out/p2.log 2>&1
rc=$?; echo "pass2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $out/p1 > $out/summary.txt
python3 tools/pmc_summary.py $out/p2 >> $out/summary.txt
cat $out/summary.txt | cut -c1-400
