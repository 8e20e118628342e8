set -o pipefail
mkdir -p gpurun_out
DX_SKINNY_FLAGS=0 PYTHONPATH=. timeout -k 10 400 python -u tools/skinny_bench.py --out gpurun_out/skinny_nont.json > gpurun_out/skinny_nont.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/skinny_nont.log; exit 1; }
cat gpurun_out/skinny_nont.log
