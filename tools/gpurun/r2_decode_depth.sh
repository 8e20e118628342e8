# decode attention: 1 vs 2 K/V chunks in flight per wave (DX_DECODE_DEPTH), numerics + microbench + headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dd
DX_DECODE_DEPTH=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k decode --timeout 120 --timeout-method thread > gpurun_out/dd/pytest.log 2>&1
rc=$?; echo "pytest depth2 rc=$rc"; tail -2 gpurun_out/dd/pytest.log; [ $rc -eq 0 ] || exit $rc
for d in 1 2; do
  DX_DECODE_DEPTH=$d timeout -k 10 300 python -u tools/microbench.py --what decode > gpurun_out/dd/micro$d.json 2> gpurun_out/dd/micro$d.err
  rc=$?; echo "micro depth=$d rc=$rc"; cat gpurun_out/dd/micro$d.json | tr -d '\n' | cut -c1-900; echo; [ $rc -eq 0 ] || exit $rc
done
for d in 2 1 2 1; do
  DX_DECODE_DEPTH=$d timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dd/bench$d.json 2> gpurun_out/dd/bench$d.err
  rc=$?; echo "bench depth=$d rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/dd/bench$d.json'));print(d['value'], d['ttft_p50_ms'], d['step_itl_p50_ms'])")"; [ $rc -eq 0 ] || exit $rc
done
