set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
timeout -k 10 500 python tools/multiturn_bench.py --model deepseek-r1-distill-llama-8b --users 32 --rounds 6 \
    --first 2000 --turn 100 --osl 150 --gpu-blocks 700 --host-blocks 0,2400 --out gpurun_out/multiturn.json \
    > gpurun_out/multiturn.log 2>&1 && \
timeout -k 10 400 python -m pytest tests/test_engine_gpu.py -q -x > gpurun_out/t_engine.log 2>&1
RC=$?
tail -3 gpurun_out/multiturn.log; tail -3 gpurun_out/t_engine.log
exit $RC
