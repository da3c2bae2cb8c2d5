# A/B of CU masks for the tracker's run-ahead detection stream (UVIO_HP_PREDETECT_CU_MASK), cfg3, alternating.
# usage: bash tools/gpu_cumask_ab.sh TAG
set -e
TAG=${1:-cum}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
(AMD_LOG_LEVEL=3 UVIO_HP_PREDETECT_CU_MASK=0,0,0,0,ffffffff,ffffffff,ffffffff,ffffffff timeout -k 10 200 python -u tools/ab_state_digest.py cfg3 6 2>&1 | grep -a "SWq\|hardware queues\|digest\|CU mask\|rror" > $O/queues_B.txt) || true
timeout -k 10 200 python -u tools/ab_state_digest.py cfg3 40 > $O/digest_A.txt 2>&1
UVIO_HP_PREDETECT_CU_MASK=0,0,0,0,ffffffff,ffffffff,ffffffff,ffffffff timeout -k 10 200 python -u tools/ab_state_digest.py cfg3 40 > $O/digest_B.txt 2>&1
for i in 1 2; do
  for v in A B C D; do
    case $v in
      A) M="" ;;
      B) M=0,0,0,0,ffffffff,ffffffff,ffffffff,ffffffff ;;
      C) M=0,ffffffff,ffffffff,ffffffff,ffffffff,ffffffff,ffffffff,ffffffff ;;
      D) M=aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa ;;
    esac
    UVIO_HP_PREDETECT_CU_MASK=$M timeout -k 10 200 python -u bench.py --workload cfg3 --steps 300 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${v}_cfg3_$i.json 2> $O/${v}_$i.err
  done
done
