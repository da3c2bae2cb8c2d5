#!/bin/bash
# Same library, same workload, twice in separate processes: the state digests must agree (device determinism).
# usage: bash tools/gpu_determinism.sh TAG FRAMES WORKLOAD...
T=$1; N=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for wl in "$@"; do
  for i in 1 2; do
    timeout -k 10 240 python -u tools/ab_state_digest.py $wl $N > $O/${wl}_$i.txt 2> $O/${wl}_$i.err || exit $?
    grep digest $O/${wl}_$i.txt
  done
done
