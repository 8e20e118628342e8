set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for gb in 1000 1400; do
  timeout -k 10 600 python -u tools/multiturn_bench.py --model deepseek-r1-distill-llama-8b --users 32 --rounds 10 --first 2000 --turn 100 --osl 150 --gpu-blocks $gb --host-blocks 0,2400 --out gpurun_out/r2_multiturn_gb$gb.json > gpurun_out/r2_multiturn_gb$gb.log 2>&1
  rc=$?; echo "gpu_blocks $gb rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$gb" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r2_multiturn_gb{sys.argv[1]}.json"))
for run in d["runs"]:
    r = run["rounds"]
    print(run["host_blocks"], "mean1+", run["ttft_mean_ms_rounds_1plus"], "r5 mean", r[5]["ttft_mean_ms"], "r5 p50", r[5]["ttft_p50_ms"], "r9 mean", r[9]["ttft_mean_ms"], "r9 p50", r[9]["ttft_p50_ms"])
PY
done
