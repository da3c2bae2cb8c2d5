# Round 6: k_feature variants (old, pass-1 unroll only, pass-2 batched loads only, both), cfg3t and cfg3 kernel traces,
# k_feature's launches split by grid size.  usage: bash tools/gpu_r06ns2.sh TAG
set -e
T=${1:-r06ns2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for wl in cfg3t cfg3; do
for lib in old p1 p2 new; do
  steps=60; [ $wl = cfg3 ] && steps=150
  (cd /tmp && UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_${wl}_$lib -o run -- python3 $R/bench.py --workload $wl --steps $steps --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_${wl}_$lib.log 2>&1)
  echo "$rep $wl $lib" >> $O/split.txt
  python tools/kernel_split.py $O/p_${wl}_$lib/run_kernel_trace.csv k_feature >> $O/split.txt
  rm -rf $O/p_${wl}_$lib
done
done
done
cat $O/split.txt
