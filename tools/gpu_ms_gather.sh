# k_ekf_MS without a chi2-gate T (the delayed initialization's update, cfg3 shape N 311 ldp 424 n 154 r 81 ldh 432):
# S from the update's own M (default) against S formed from P (UVIO_HP_MS_FROM_P=1); checksums must agree.
# usage: bash tools/gpu_ms_gather.sh [TAG]
set -e
O=gpurun_out/${1:-r04w}; mkdir -p $O
B=$GRAFT_REPO_ROOT/build/bench_small_chain
timeout -k 10 60 $B 300 311 424 154 81 432 0 > $O/gather.txt
UVIO_HP_MS_FROM_P=1 timeout -k 10 60 $B 300 311 424 154 81 432 0 > $O/from_p.txt
timeout -k 10 60 $B 300 314 424 223 82 432 1 > $O/slam_tall.txt
head -5 $O/*.txt
