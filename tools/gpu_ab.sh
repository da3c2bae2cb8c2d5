# A/B of the current library against another build (UVIO_HP_LIB) on one box: bench lines per workload.
# usage: bash tools/gpu_ab.sh OTHER_LIB OUTDIR workload...
set -e
R=$GRAFT_REPO_ROOT
B=$1; O=$R/gpurun_out/$2; shift 2
cd $R && mkdir -p $O
for wl in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $wl --cpu-frames 0 > $O/${wl}_new.json 2> $O/${wl}_new.err
  UVIO_HP_LIB=$R/$B timeout -k 10 300 python -u bench.py --workload $wl --cpu-frames 0 > $O/${wl}_old.json 2> $O/${wl}_old.err
done
