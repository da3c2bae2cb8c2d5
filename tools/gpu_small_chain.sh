# Isolated timings of launch_trsm_lt / launch_ekf_phaseA (tools/bench_small_chain.cpp), default and split M / S
# usage: bash tools/gpu_small_chain.sh [TAG]
set -e
O=gpurun_out/${1:-r04t}; mkdir -p $O
B=$GRAFT_REPO_ROOT/build/bench_small_chain
timeout -k 10 60 $B 300 > $O/default.txt
UVIO_HP_MS_SPLIT=1 timeout -k 10 60 $B 300 > $O/split.txt
head -3 $O/*.txt
