set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-dr}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -rf --timeout 200 --timeout-method thread -k "sample_draws_kernels" > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "draws exact|passed|failed" gpurun_out/tests_$TAG.log
