#!/bin/bash
# Host-section profiles (UVIO_HP_HOST_PROF=1: hprof lines on stderr) of bench workloads.
# usage: bash tools/gpu_hostprof.sh TAG WORKLOAD...
set -e
TAG=${1:-dev}
shift
O=gpurun_out/$TAG
mkdir -p $O
for wl in "$@"; do
  UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 100 --cpu-frames 0 --no-host-feed \
    --msckf-load-steps 0 > $O/${wl}_bench.json 2> $O/${wl}.err
  grep hprof $O/${wl}.err | sort -k3 -n -r | head -14
  python -c "import json; d = json.load(open('$O/${wl}_bench.json')); print('$wl', round(d['value'], 1), d['unit'])"
done
