# selected GPU tests, then an A/B against another library build.   usage: bash tools/gpu_test_ab.sh TAG "pytest -k" OTHER_LIB REPEATS workload...
set -e
TAG=$1; KEXPR=$2; B=$3; N=$4; shift 4
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" > $O/gpu_tests.log 2>&1
bash tools/gpu_ab.sh $B ${TAG}_ab $N "$@"
