set -o pipefail
mkdir -p gpurun_out
python -c "import dynamo_exp_amd.build_native as b; b.build_all()" > /dev/null
run() { # name waves steps warmup
  DX_PREFILL_WAVES=$2 timeout -k 10 400 python bench.py --steps $3 --warmup $4 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { echo BENCH_FAIL $1; tail gpurun_out/ab_$1.err; exit 1; }
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));print(d['value'],d['ttft_p50_ms'],d['ms_per_step'],d['config']['itl_p50_ms'],d['config']['decode_steps'],d['config']['mixed_steps'])")"
  grep "steady-state" gpurun_out/ab_$1.err
}
run v91_500 91 500 200 && run v81_500 81 500 200 && run v91_60 91 60 10 && run v91_20 91 20 5
