set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err && cat gpurun_out/bench_n1.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ss -o ss -- python3 $R/bench.py --steps 200 --warmup 50 > $R/gpurun_out/prof_ss.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_ss.log; exit 1; }
cd $R
DB=$(find gpurun_out/prof_ss -name "*.db" | head -1)
python tools/prof_summary.py $DB 30 > gpurun_out/prof_ss_summary.txt
python tools/prof_summary.py $DB --busy 9 >> gpurun_out/prof_ss_summary.txt
head -16 gpurun_out/prof_ss_summary.txt
tail -1 gpurun_out/prof_ss_summary.txt
