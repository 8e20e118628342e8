set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof2
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py tests/test_multimodal.py -x -q > gpurun_out/t_eng2.log 2>&1 || { echo ENGINE_TEST_FAIL; tail -40 gpurun_out/t_eng2.log; exit 1; }
tail -1 gpurun_out/t_eng2.log
timeout -k 10 400 python bench.py > gpurun_out/b_on.json 2> gpurun_out/b_on.err || { echo BENCH_FAIL; tail -20 gpurun_out/b_on.err; exit 1; }
echo "overlap=1 $(cat gpurun_out/b_on.json)"
DX_OVERLAP_DECODE_ATTN=0 timeout -k 10 400 python bench.py > gpurun_out/b_off.json 2> gpurun_out/b_off.err || { echo BENCH_FAIL; tail -20 gpurun_out/b_off.err; exit 1; }
echo "overlap=0 $(cat gpurun_out/b_off.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2 -o bench -- python3 $R/bench.py --steps 200 --warmup 100 > $R/gpurun_out/prof2/bench.json 2> $R/gpurun_out/prof2/bench.err || { echo PROF_FAIL; tail -5 $R/gpurun_out/prof2/bench.err; exit 1; }
ls $R/gpurun_out/prof2
