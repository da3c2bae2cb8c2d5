#!/bin/bash
# Host-ISA A/B: state digests of both libraries (must agree) and alternating bench runs.
# usage: bash tools/gpu_isa_ab.sh TAG   (build/abprev/libuvio_hp_prev.so = the other build)
set -e
T=${1:-isa}
O=gpurun_out/$T
mkdir -p $O
for wl in cfg3 cfg5; do
  timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_new.txt 2> $O/digest_${wl}_new.err
  UVIO_HP_LIB=build/abprev/libuvio_hp_prev.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_old.txt 2> $O/digest_${wl}_old.err
  cat $O/digest_${wl}_new.txt $O/digest_${wl}_old.txt
done
bash tools/gpu_env_ab.sh UVIO_HP_LIB=build/abprev/libuvio_hp_prev.so $T 4 100 cfg5 cfg3
python tools/ab_summary.py $O 2>/dev/null || true
