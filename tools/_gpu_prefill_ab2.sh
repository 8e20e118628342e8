set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
for w in 83 81; do
  DX_PREFILL_WAVES=$w timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k prefill > gpurun_out/t_pf$w.log 2>&1 || { echo PREFILL_TEST_FAIL $w; tail -30 gpurun_out/t_pf$w.log; exit 1; }
  echo "waves=$w tests: $(tail -1 gpurun_out/t_pf$w.log)"
  DX_PREFILL_WAVES=$w timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/mb_pf$w.json 2> gpurun_out/mb_pf$w.err || { echo MB_FAIL; tail gpurun_out/mb_pf$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/mb_pf$w.json'));print('waves=$w', {k:v for k,v in d.items() if 'prefill' in k})"
done
for w in 83 81; do
  DX_OVERLAP_DECODE_ATTN=0 DX_PREFILL_WAVES=$w timeout -k 10 400 python bench.py > gpurun_out/b_pf$w.json 2> gpurun_out/b_pf$w.err || { echo BENCH_FAIL; tail -20 gpurun_out/b_pf$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_pf$w.json'));print('bench waves=$w', d['value'], d['ttft_p50_ms'], d['config']['itl_p50_ms'])"
done
