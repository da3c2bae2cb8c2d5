#!/bin/bash
# Run microbenchmark binaries (built on the CPU side) one after another, each under its own time limit.
# usage: bash tools/gpu_ab_bins.sh TAG BIN...   (outputs gpurun_out/TAG/<bin>.txt)
set -o pipefail
T=${1:-ab}
shift
O=gpurun_out/$T
mkdir -p $O
for b in "$@"; do
  n=$(basename $b)
  timeout -k 10 120 $b > $O/$n.txt 2>&1 || { echo "$b failed"; exit 1; }
  echo "== $n"; cat $O/$n.txt
done
