# prosody tests then bench (iteration loop)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-pi}
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_prosody.py > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/tests_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --prosody --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
grep -o '"roofline.*' gpurun_out/bench_$TAG.log | cut -c1-200
