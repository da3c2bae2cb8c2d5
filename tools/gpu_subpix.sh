#!/bin/bash
# k_subpix A/B (previous kernel vs this tree's, same points, digests must agree) + the tracker bit-exact tests.
# usage: bash tools/gpu_subpix.sh TAG   (build/bench_subpix{,_old} built beforehand on the CPU side)
set -o pipefail
T=${1:-sp}
O=gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  timeout -k 10 60 ./build/bench_subpix_old 100 > $O/old_$i.txt 2>&1 || exit 1
  timeout -k 10 60 ./build/bench_subpix 100 > $O/new_$i.txt 2>&1 || exit 1
done
cat $O/old_*.txt $O/new_*.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_track.py > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
exit $rc
