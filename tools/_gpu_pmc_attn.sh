set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/pmc -o attn -- python3 $R/tools/microbench.py --what attn > $R/gpurun_out/pmc/mb.log 2>&1
ls -R $R/gpurun_out/pmc | head -20
