set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/g1
timeout -k 5 60 ./build/bench_sync 0 > gpurun_out/g1/sync.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lockstep_images or updaters or stereo or mono or smoke or cfg" > gpurun_out/g1/tests.log 2>&1
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --steps 300 --cpu-frames 0 > gpurun_out/g1/b.json 2> gpurun_out/g1/b.err
bash tools/gpu_prof.sh g1 cfg2
