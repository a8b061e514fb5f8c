# Self-attention A/B: beam/sampling parity tests (default kernel and MWX_SELF_UB=4),
# then beam-5 and greedy bench legs for both, and a beam profile of each.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-sab}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "fallback or beam or draws or greedy" > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
MWX_SELF_UB=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "fallback or beam or draws or greedy" > gpurun_out/tests_${TAG}_ub4.log 2>&1; echo "ub4 tests rc=$?"
tail -3 gpurun_out/tests_${TAG}_ub4.log
for v in 8 4; do
  MWX_SELF_UB=$v timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5_ub$v.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5_ub$v.log; exit 1; }
  echo "ub$v beam: $(tail -1 gpurun_out/bench_${TAG}_b5_ub$v.log | cut -c80-140)"
  MWX_SELF_UB=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_g_ub$v.log 2>&1 || { echo "greedy bench failed"; exit 1; }
  echo "ub$v greedy: $(tail -1 gpurun_out/bench_${TAG}_g_ub$v.log | cut -c80-140)"
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_ub8 -o beam -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_ub8.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
