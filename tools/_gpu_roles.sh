set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/role_bench.py --agg 2600 > gpurun_out/roles.json 2> gpurun_out/roles.err || { echo ROLE_FAIL; tail -30 gpurun_out/roles.err; exit 1; }
cat gpurun_out/roles.json
timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/mb_attn.json 2> gpurun_out/mb_attn.err && timeout -k 10 300 python tools/microbench.py --what decode > gpurun_out/mb_dec.json 2> gpurun_out/mb_dec.err && cat gpurun_out/mb_attn.json gpurun_out/mb_dec.json
