set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
DX_PREFILL_WAVES=91 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "prefill" > gpurun_out/t_pf91.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t_pf91.log; exit 1; }
tail -2 gpurun_out/t_pf91.log
for w in 81 91; do
  DX_PREFILL_WAVES=$w timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/mb_pf$w.json 2> gpurun_out/mb_pf$w.err || { echo MB_FAIL; tail gpurun_out/mb_pf$w.err; exit 1; }
done
for w in 91 81; do
  DX_PREFILL_WAVES=$w timeout -k 10 400 python bench.py --steps 400 --warmup 150 > gpurun_out/b_pf$w.json 2> gpurun_out/b_pf$w.err || { echo BENCH_FAIL; tail gpurun_out/b_pf$w.err; exit 1; }
done
grep prefill gpurun_out/mb_pf81.json gpurun_out/mb_pf91.json
cat gpurun_out/b_pf91.json gpurun_out/b_pf81.json
