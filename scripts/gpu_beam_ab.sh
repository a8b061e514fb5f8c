# GPU parity tests, then beam-5 bench: XCD-co-scheduled per-row cross-attn vs grouped kernel; profile.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 600 python -u -m pytest tests -m gpu ${PYTEST_K:+-k "$PYTEST_K"} -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_b5.log | cut -c1-200
MWX_XATTN8=1 timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5g.log 2>&1 || { echo "beam bench grouped failed"; tail -20 gpurun_out/bench_${TAG}_b5g.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_b5g.log | cut -c1-200
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o beam -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
