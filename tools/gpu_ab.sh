# A/B of the current library against another build (UVIO_HP_LIB) on one box, alternating runs so box
# drift hits both arms alike.  usage: bash tools/gpu_ab.sh OTHER_LIB OUTDIR REPEATS workload...
set -e
R=$GRAFT_REPO_ROOT
B=$1; O=$R/gpurun_out/$2; N=$3; shift 3
cd $R && mkdir -p $O
for wl in "$@"; do
  for i in $(seq 1 $N); do
    # ABBA: the arm that runs first alternates, so an order effect hits both arms alike
    if [ $((i % 2)) = 1 ]; then
      timeout -k 10 300 python -u bench.py --workload $wl --cpu-frames 0 > $O/${wl}_new_$i.json 2> $O/${wl}_new_$i.err
      UVIO_HP_AB_OLD=1 UVIO_HP_LIB=$R/$B timeout -k 10 300 python -u bench.py --workload $wl --cpu-frames 0 > $O/${wl}_old_$i.json 2> $O/${wl}_old_$i.err
    else
      UVIO_HP_AB_OLD=1 UVIO_HP_LIB=$R/$B timeout -k 10 300 python -u bench.py --workload $wl --cpu-frames 0 > $O/${wl}_old_$i.json 2> $O/${wl}_old_$i.err
      timeout -k 10 300 python -u bench.py --workload $wl --cpu-frames 0 > $O/${wl}_new_$i.json 2> $O/${wl}_new_$i.err
    fi
  done
done
python tools/ab_summary.py $O > $O/summary.txt
