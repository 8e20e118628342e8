set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gemm.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_skinny.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/t_skinny.log; exit 1; }
tail -1 gpurun_out/t_skinny.log
timeout -k 10 500 python -u bench.py --gemm-report gpurun_out/gemm_report.json > gpurun_out/b_sk1.json 2> gpurun_out/b_sk1.err || { echo BENCH_FAIL; tail -20 gpurun_out/b_sk1.err; exit 1; }
echo "skinny=1 $(cat gpurun_out/b_sk1.json)"
DX_SKINNY=0 timeout -k 10 500 python -u bench.py > gpurun_out/b_sk0.json 2> gpurun_out/b_sk0.err || { echo BENCH_FAIL; tail -20 gpurun_out/b_sk0.err; exit 1; }
echo "skinny=0 $(cat gpurun_out/b_sk0.json)"
python -c "
import json; r=json.load(open('gpurun_out/gemm_report.json'))
for x in r: print(x)
"
