# sampling / beam parity tests + beam-5 bench and profile
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-bq}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "fallback or beam or draws" > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_b5.log | cut -c1-200
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_b5 -o beam -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_b5.log 2>&1 || { echo "beam prof failed"; exit 1; }
echo done
