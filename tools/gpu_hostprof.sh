# host section times (UVIO_HP_HOST_PROF) of the cfg2 bench.   usage: bash tools/gpu_hostprof.sh TAG
set -e
TAG=${1:-hp}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --steps 300 --cpu-frames 0 > $O/hp.json 2> $O/hp.err
