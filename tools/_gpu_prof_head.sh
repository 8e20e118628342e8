set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o head -- python3 $R/bench.py --steps 300 --warmup 150 > $R/gpurun_out/prof_head.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_head.log; exit 1; }
cd $R
DB=$(find gpurun_out/prof_head -name "*.db" | head -1)
python tools/prof_summary.py $DB 30 > gpurun_out/prof_head_summary.txt
python tools/prof_summary.py $DB --busy 6 >> gpurun_out/prof_head_summary.txt
head -16 gpurun_out/prof_head_summary.txt
tail -1 gpurun_out/prof_head_summary.txt
grep '"metric"' gpurun_out/prof_head.log | cut -c1-400
