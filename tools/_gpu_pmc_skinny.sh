set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcsk
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/pmcsk/p1 -o sk -- python3 $R/tools/skinny_pmc_driver.py > $R/gpurun_out/pmcsk/p1.log 2>&1 || { echo P1_FAIL; tail -20 $R/gpurun_out/pmcsk/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d $R/gpurun_out/pmcsk/p2 -o sk -- python3 $R/tools/skinny_pmc_driver.py > $R/gpurun_out/pmcsk/p2.log 2>&1 || { echo P2_FAIL; tail -20 $R/gpurun_out/pmcsk/p2.log; exit 1; }
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcsk/p1 > gpurun_out/pmcsk/summary1.txt 2>&1; python3 tools/pmc_summary.py gpurun_out/pmcsk/p2 > gpurun_out/pmcsk/summary2.txt 2>&1; cat gpurun_out/pmcsk/summary1.txt gpurun_out/pmcsk/summary2.txt
