# scratch measurement recipe for one gpurun call (outputs under gpurun_out/q1)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/q1
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u tools/stage_times.py cfg4 30 1 > $O/st4.log 2>&1
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u tools/stage_times.py cfg2 100 1 > $O/st2.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-frames 0 > $O/b2.json 2> $O/b2.err
timeout -k 10 300 python -u bench.py --workload cfg4 --cpu-frames 0 > $O/b4.json 2> $O/b4.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --steps 200 --warmup 50 --cpu-frames 0 > $O/p2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p4 -o run -- python3 $R/bench.py --workload cfg4 --steps 30 --warmup 20 --cpu-frames 0 > $O/p4.log 2>&1
