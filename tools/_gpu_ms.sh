set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out
for k in 2 4; do
  DX_MULTI_STEP=$k timeout -k 10 300 python -u bench.py > gpurun_out/ms_$k.json 2> gpurun_out/ms_$k.err || { echo BENCH_FAIL $k; tail -20 gpurun_out/ms_$k.err; exit 1; }
  echo "ms=$k $(cat gpurun_out/ms_$k.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pb -o pb -- python3 $R/bench.py --steps 300 --warmup 150 > $R/gpurun_out/prof_pb.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_pb.log; exit 1; }
cd $R
python tools/prof_summary.py $(find gpurun_out/prof_pb -name "*.db" | head -1) 24 > gpurun_out/prof_pb_summary.txt
python tools/prof_summary.py $(find gpurun_out/prof_pb -name "*.db" | head -1) --busy 6 >> gpurun_out/prof_pb_summary.txt
rm -rf gpurun_out/prof_pb
cat gpurun_out/prof_pb_summary.txt
