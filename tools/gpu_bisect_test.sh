#!/bin/bash
# Run one GPU test against several library builds (UVIO_HP_LIB); a failing assertion moves on to the next build,
# a timeout / abort / crash ends the script.  usage: bash tools/gpu_bisect_test.sh TAG TEST LIB...
T=$1; TEST=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for lib in "$@"; do
  n=$(basename $lib .so)
  UVIO_HP_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread "$TEST" > $O/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log)"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then exit $rc; fi
done
exit 0
