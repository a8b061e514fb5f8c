# GPU iteration: parity tests, bench (large-v3, B=32), kernel-trace profile.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 600 python -m pytest tests -m gpu -q -rf --timeout 300 > gpurun_out/tests_$TAG.log 2>&1; echo "tests rc=$?" >> gpurun_out/tests_$TAG.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o large -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
