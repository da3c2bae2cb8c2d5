# LDL lag-1 microbenchmark + propagation tests + cfg5/cfg5i host profiles.  usage: bash tools/gpu_r05m.sh TAG
set -e
TAG=${1:-dev}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 120 ./build/bench_fact_lag > $O/fact_lag.txt 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "uwb or cfg5 or lockstep_images or fd or propagat" > $O/gpu_tests.log 2>&1
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload cfg5 --steps 60 --cpu-frames 0 > $O/${TAG}_cfg5_bench.json 2> $O/cfg5.err
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload cfg5i --steps 60 --cpu-frames 0 --no-host-feed > $O/${TAG}_cfg5i_bench.json 2> $O/cfg5i.err
