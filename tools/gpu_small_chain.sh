# Isolated timings of launch_trsm_lt / launch_ekf_phaseA (tools/bench_small_chain.cpp), default and split M / S
# usage: bash tools/gpu_small_chain.sh [TAG]
set -e
O=gpurun_out/${1:-r04t}; mkdir -p $O
B=$GRAFT_REPO_ROOT/build/bench_small_chain
timeout -k 10 60 $B 300 > $O/default.txt
UVIO_HP_MS_SPLIT=1 timeout -k 10 60 $B 300 > $O/split.txt
head -5 $O/*.txt
export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- $B 300 > /dev/null
cd $GRAFT_REPO_ROOT && find $O/prof -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-8
