set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prefix_stress.py --conc 12 --requests 300 > gpurun_out/stress1.log 2>&1; echo rc=$?; tail -3 gpurun_out/stress1.log
timeout -k 10 300 python -u tools/prefix_stress.py --conc 16 --requests 300 --blocks 300 > gpurun_out/stress2.log 2>&1; echo rc=$?; tail -3 gpurun_out/stress2.log
