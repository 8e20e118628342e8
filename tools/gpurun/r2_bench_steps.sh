set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/steps
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -1 gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/steps -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/steps/bench.json 2> gpurun_out/steps/bench.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
k=$(find gpurun_out/steps -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py "$k" 10 > gpurun_out/steps/breakdown.txt 2>&1; cat gpurun_out/steps/breakdown.txt
python3 tools/prof_summary.py "$k" 30 > gpurun_out/steps/summary.txt 2>&1
rm -f "$k"
