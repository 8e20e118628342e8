# single-GPU capacities of the disaggregated roles at the current kernels (prefill-only engine at the
# prefill ranks' 16384-token budget; decode-only engine at the decode ranks' 256 streams)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/roles
timeout -k 10 600 python -u tools/role_bench.py --role both --budget 16384 --agg 3085 > gpurun_out/roles/roles.txt 2> gpurun_out/roles/roles.err
rc=$?; echo "roles rc=$rc"; cat gpurun_out/roles/roles.txt; tail -3 gpurun_out/roles/roles.err; exit $rc
