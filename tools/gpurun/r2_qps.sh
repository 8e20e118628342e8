# Open-loop (Poisson) TTFT at fixed QPS on one GPU (BASELINE metric's "p50 TTFT at fixed QPS"),
# then a rocprofv3 --stats profile of the closed-loop headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qps gpurun_out/prof
for q in 8 14 18 20; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --qps $q > gpurun_out/qps/q$q.json 2> gpurun_out/qps/q$q.err
  rc=$?; echo "qps=$q rc=$rc $(tail -1 gpurun_out/qps/q$q.json | cut -c1-400)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > gpurun_out/prof/breakdown.txt 2>&1; cat gpurun_out/prof/breakdown.txt
python3 tools/prof_summary.py "$k" 30 > gpurun_out/prof/summary.txt 2>&1
rm -f "$k"
