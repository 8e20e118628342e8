set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/pmc1 $R/gpurun_out/pmc2 $R/gpurun_out/pmc3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/pmc1 -o p1 -- python3 $R/tools/microbench.py --what attn > $R/gpurun_out/pmc1/run.log 2>&1 || { echo PMC1_FAIL; tail -5 $R/gpurun_out/pmc1/run.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc2 -o p2 -- python3 $R/tools/microbench.py --what attn > $R/gpurun_out/pmc2/run.log 2>&1 || { echo PMC2_FAIL; tail -5 $R/gpurun_out/pmc2/run.log; exit 1; }
cd $R
ls -R gpurun_out/pmc1 | head; python tools/pmc_summary.py gpurun_out/pmc1 | head -8; python tools/pmc_summary.py gpurun_out/pmc2 | head -8
