# PMC passes (one counter group per run, as the MI355X guide prescribes): FETCH_SIZE, WRITE_SIZE, FP64 MFMA work,
# per workload -> profiles/TAG_pmc_traffic_WL.json.   usage: bash tools/gpu_pmc.sh TAG workload...
set -e
TAG=${1:-dev}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O profiles
export TMPDIR=/tmp
for wl in "$@"; do
  steps=100
  case $wl in cfg4|cfg5) steps=20 ;; cfg4i|cfg5i) steps=50 ;; esac
  B="$R/bench.py --workload $wl --steps $steps --warmup 20 --cpu-frames 0 --no-host-feed --msckf-load-steps 0"
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_$wl -o run -- python3 $B > $O/pf_$wl.log 2>&1)
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw_$wl -o run -- python3 $B > $O/pw_$wl.log 2>&1)
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pm_$wl -o run -- python3 $B > $O/pm_$wl.log 2>&1)
  python tools/pmc_summary.py $O/pf_$wl/run_counter_collection.csv $O/pw_$wl/run_counter_collection.csv profiles/${TAG}_pmc_traffic_$wl.json $O/pm_$wl/run_counter_collection.csv
  cp profiles/${TAG}_pmc_traffic_$wl.json $O/
  rm -rf $O/pf_$wl $O/pw_$wl $O/pm_$wl
done
