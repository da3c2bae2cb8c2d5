# A/B of one environment switch on one box (e.g. UVIO_HP_NO_CHAIN=1), alternating runs so box drift hits both
# arms alike.  usage: bash tools/gpu_env_ab.sh VAR=VALUE OUTDIR REPEATS STEPS workload...
set -e
R=$GRAFT_REPO_ROOT
E=$1; O=$R/gpurun_out/$2; N=$3; S=$4; shift 4
cd $R && mkdir -p $O
for wl in "$@"; do
  for i in $(seq 1 $N); do
    if [ $((i % 2)) = 1 ]; then
      timeout -k 10 300 python -u bench.py --workload $wl --steps $S --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_new_$i.json 2> $O/${wl}_new_$i.err
      env $E timeout -k 10 300 python -u bench.py --workload $wl --steps $S --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_old_$i.json 2> $O/${wl}_old_$i.err
    else
      env $E timeout -k 10 300 python -u bench.py --workload $wl --steps $S --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_old_$i.json 2> $O/${wl}_old_$i.err
      timeout -k 10 300 python -u bench.py --workload $wl --steps $S --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_new_$i.json 2> $O/${wl}_new_$i.err
    fi
  done
done
python tools/ab_summary.py $O > $O/summary.txt
