# LK A/B on one MI355X: microbenchmark of the previous and the current kernel (cycle breakdown + results digest),
# the tracker's bit-exactness tests, then the driver-form cfg3 line and its kernel-trace summary.
# usage: bash tools/gpu_lk_ab.sh TAG   (build/bench_lk_old, build/bench_lk_new built beforehand)
set -e
TAG=${1:-dev}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for n in 400 800; do
  timeout -k 10 60 ./build/bench_lk_old $n > $O/lk_old_$n.txt 2>&1
  timeout -k 10 60 ./build/bench_lk_new $n > $O/lk_new_$n.txt 2>&1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bit_exact or predetect or lockstep_images" > $O/gpu_tests.log 2>&1
bash tools/gpu_new.sh $TAG
