# Decode row-group sweep: parity tests, then bench at MWX_DECODE_GROUPS = 1, 2, 4.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-groups}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
for G in ${GROUPS_LIST:-1 2 4}; do
  MWX_DECODE_GROUPS=$G timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_g$G.log 2>&1 || { echo "bench G=$G failed"; tail -20 gpurun_out/bench_${TAG}_g$G.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_g$G.log | cut -c1-200
done
echo done
