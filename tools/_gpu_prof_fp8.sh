set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fp8 -o fp8 -- python3 $R/bench.py --quantization fp8 --steps 200 --warmup 50 > $R/gpurun_out/prof_fp8.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_fp8.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec -o dec -- python3 $R/tools/role_bench.py --role decode --steps 60 > $R/gpurun_out/prof_dec.log 2>&1 || { echo PROF2_FAIL; tail -20 $R/gpurun_out/prof_dec.log; exit 1; }
cd $R
python tools/prof_summary.py $(find gpurun_out/prof_fp8 -name "*.db" | head -1) 20 > gpurun_out/prof_fp8_summary.txt
python tools/prof_summary.py $(find gpurun_out/prof_fp8 -name "*.db" | head -1) --busy 6 >> gpurun_out/prof_fp8_summary.txt
python tools/prof_summary.py $(find gpurun_out/prof_dec -name "*.db" | head -1) 20 > gpurun_out/prof_dec_summary.txt
python tools/prof_summary.py $(find gpurun_out/prof_dec -name "*.db" | head -1) --busy 1.2 >> gpurun_out/prof_dec_summary.txt
head -14 gpurun_out/prof_fp8_summary.txt; tail -1 gpurun_out/prof_fp8_summary.txt; head -12 gpurun_out/prof_dec_summary.txt; tail -1 gpurun_out/prof_dec_summary.txt
