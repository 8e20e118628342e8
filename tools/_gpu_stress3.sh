set -o pipefail
mkdir -p gpurun_out
for q in 2 1; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/prefix_stress.py --conc 12 --requests 400 --slow-s 1.0 > gpurun_out/stressA_q$q.log 2>&1 &
A=$!
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/prefix_stress.py --conc 12 --requests 400 --slow-s 1.0 > gpurun_out/stressB_q$q.log 2>&1 &
B=$!
wait $A; RA=$?
wait $B; RB=$?
echo "queues=$q rc $RA $RB slow: $(grep -c SLOW gpurun_out/stressA_q$q.log) $(grep -c SLOW gpurun_out/stressB_q$q.log)"
tail -n1 gpurun_out/stressA_q$q.log
[ $RA -eq 0 ] && [ $RB -eq 0 ] || exit 1
done
