set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --trace-steps > gpurun_out/r2_bench_v.json 2> gpurun_out/r2_bench_v.err
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r2_bench_v.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/prof/bench_prof.json 2> gpurun_out/prof/bench_prof.err
rc=$?; echo "rocprof rc=$rc"
f=$(ls gpurun_out/prof/*/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
echo "stats: $f"; head -30 "$f" > gpurun_out/prof/kernel_stats_head.csv
k=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); echo "trace: $k"
python3 tools/prof_summary.py "$k" 30 > gpurun_out/prof/summary.txt 2>&1; head -40 gpurun_out/prof/summary.txt
rm -f "$k"
