set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/prefix_stress.py --conc 12 --requests 600 --slow-s 1.0 > gpurun_out/stressA.log 2>&1 &
A=$!
timeout -k 10 400 python -u tools/prefix_stress.py --conc 12 --requests 600 --slow-s 1.0 > gpurun_out/stressB.log 2>&1 &
B=$!
wait $A; RA=$?
wait $B; RB=$?
echo rc $RA $RB
grep -c SLOW gpurun_out/stressA.log gpurun_out/stressB.log || true
tail -1 gpurun_out/stressA.log gpurun_out/stressB.log
grep SLOW gpurun_out/stressA.log | head -3
