set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b2
for i in 1 2; do
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b2/bench$i.json 2> gpurun_out/b2/bench$i.err
  rc=$?; echo "bench $i rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/b2/bench$i.json'));print(d['value'], d['ttft_p50_ms'], d['elapsed_s'])")"; [ $rc -eq 0 ] || exit $rc
done
