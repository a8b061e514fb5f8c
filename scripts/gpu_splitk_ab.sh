# Split-K decode GEMM row-block A/B for M > 64 (beam rows): MWX_SPLITK_MT = 4 / 2 / 3;
# beam / best-of parity tests with MT = 2, beam-5 legs, beam profile with MT = 2.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-spab}
MWX_SPLITK_MT=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "fallback or beam or draws" > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for v in 4 2 3 2 4; do
  MWX_SPLITK_MT=$v timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5_mt$v.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5_mt$v.log; exit 1; }
  echo "mt$v beam: $(tail -1 gpurun_out/bench_${TAG}_b5_mt$v.log | cut -c80-140)"
done
cd /tmp && MWX_SPLITK_MT=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o beam -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
