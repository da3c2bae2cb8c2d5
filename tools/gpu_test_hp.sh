# selected GPU tests, then the cfg2 host-section profile.   usage: bash tools/gpu_test_hp.sh TAG "pytest -k expr"
set -e
TAG=${1:-dev}; KEXPR=${2:-parity}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" > $O/gpu_tests.log 2>&1
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --steps 300 --cpu-frames 0 > $O/hp.json 2> $O/hp.err
