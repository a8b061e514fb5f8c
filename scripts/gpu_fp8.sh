# MX-fp8 compute mode: parity tests, bench legs (greedy, fp8), encoder-GEMM profile.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-fp8}
timeout -k 10 600 python -u -m pytest tests -m gpu ${PYTEST_K:+-k "$PYTEST_K"} -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp8 > gpurun_out/bench_${TAG}.log 2>&1 || { echo "fp8 bench failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-200
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o fp8 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --fp8 --decode-steps 8 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
