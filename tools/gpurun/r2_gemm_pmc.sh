set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 tools/gemm_pmc_driver.py > gpurun_out/pmc/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 tools/gemm_pmc_driver.py > gpurun_out/pmc/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc/p3 -o p3 --output-format csv -- python3 tools/gemm_pmc_driver.py > gpurun_out/pmc/p3.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc/p1 > gpurun_out/pmc/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc/p2 >> gpurun_out/pmc/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc/p3 >> gpurun_out/pmc/summary.txt
cat gpurun_out/pmc/summary.txt
