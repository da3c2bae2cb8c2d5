# One GPU call's worth of measurements while iterating: LDL slot bench, determinism, chi2 phases, host profiles
# of cfg4 / cfg3, the GPU test suite, FETCH calibration and the N=2 rehearsal.
# usage: bash tools/gpu_round_check.sh TAG
TAG=${1:-chk}; O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 60 build/bench_wave_slots > $O/wave_slots.txt 2>&1 &&
timeout -k 10 300 python -u tools/diag_determinism.py 60 > $O/determinism.log 2>&1 &&
timeout -k 10 200 python -u tools/feat_phases.py cfg3 > $O/feat_phases_cfg3.txt 2>&1 &&
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload cfg4 --steps 300 --cpu-frames 0 --no-host-feed > $O/hp_cfg4.json 2> $O/hp_cfg4.err &&
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload cfg3 --steps 300 --cpu-frames 0 --no-host-feed > $O/hp_cfg3.json 2> $O/hp_cfg3.err &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?
cat $O/wave_slots.txt; tail -3 $O/determinism.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_fetch_calib.sh $TAG/fc &&
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse --steps 30 --warmup 5 --sharded-steps 20 > $O/rehearse2.json 2> $O/rehearse2.err
