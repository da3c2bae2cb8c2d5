# ldl_wave_inv option bits on one MI355X (tools/bench_fact_opt.hip).  usage: bash tools/gpu_fact_opt.sh TAG
set -e
TAG=${1:-dev}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 120 ./build/bench_fact_opt > $O/fact_opt.txt 2>&1
