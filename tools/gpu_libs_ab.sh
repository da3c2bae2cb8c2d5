#!/bin/bash
# Alternating bench runs of several library builds on one box (UVIO_HP_LIB), round robin so drift hits all alike.
# usage: bash tools/gpu_libs_ab.sh TAG REPEATS STEPS WORKLOAD LIB...
set -e
T=$1; N=$2; S=$3; WL=$4; shift 4
O=gpurun_out/$T
mkdir -p $O
for i in $(seq 1 $N); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    UVIO_HP_LIB=$lib timeout -k 10 300 python -u bench.py --workload $WL --steps $S --cpu-frames 0 --no-host-feed \
      --msckf-load-steps 0 > $O/${WL}_${n}_$i.json 2> $O/${WL}_${n}_$i.err
  done
done
python - "$O" "$WL" "$@" <<'PY'
import json, os, sys, statistics
o, wl, libs = sys.argv[1], sys.argv[2], sys.argv[3:]
for lib in libs:
    n = os.path.basename(lib)[:-3]
    v = [json.load(open(os.path.join(o, f)))["value"] for f in sorted(os.listdir(o)) if f.startswith(wl + "_" + n + "_") and f.endswith(".json")]
    print("%-6s %-20s median %7.1f  %s" % (wl, n, statistics.median(v), " ".join("%.1f" % x for x in v)))
PY
