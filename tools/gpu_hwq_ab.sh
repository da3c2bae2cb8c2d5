# A/B of the HIP runtime's hardware-queue count (GPU_MAX_HW_QUEUES 4, the box default, against 8): do the tracker's
# detection stream and the engine's streams share a queue?  First the runtime's own stream -> queue log of a short
# cfg3 run.  usage: bash tools/gpu_hwq_ab.sh TAG
set -e
TAG=${1:-hwq}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
(AMD_LOG_LEVEL=4 timeout -k 10 200 python -u tools/ab_state_digest.py cfg3 6 2>&1 | grep -a "SWq\|hardware queues\|digest" > $O/queues.txt) || true
for i in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --workload cfg3 --steps 300 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/q${q}_cfg3_$i.json 2> /dev/null
  done
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --workload cfg3t --steps 100 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/q${q}_cfg3t.json 2> /dev/null
done
