# LK microbenchmark over prebuilt variants (build/bench_lk_*), 800 and 400 points.  usage: bash tools/gpu_lk_variants.sh TAG
set -e
TAG=${1:-dev}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for b in build/bench_lk_*; do
  n=$(basename $b)
  for np in 800 400; do timeout -k 10 60 ./$b $np >> $O/$n.txt 2>&1; done
done
