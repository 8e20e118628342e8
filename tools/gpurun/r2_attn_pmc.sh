set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/apmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/apmc/p1 -o p1 --output-format csv -- python3 tools/microbench.py --what attn > gpurun_out/apmc/p1.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/apmc/p1 > gpurun_out/apmc/summary.txt
grep -i "prefill_attn\|decode_attn" gpurun_out/apmc/summary.txt
