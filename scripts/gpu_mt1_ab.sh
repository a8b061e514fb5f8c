# Greedy decode GEMM row-block A/B: 16-row blocks (MWX_DEC_MT1=1) vs the default
# for M <= 64; greedy parity tests with MT1, greedy legs both ways.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-mt1}
MWX_DEC_MT1=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "greedy or batch or long_form" > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for v in 0 1 0 1; do
  MWX_DEC_MT1=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_g_$v.log 2>&1 || { echo "greedy bench failed"; exit 1; }
  echo "mt1=$v greedy: $(tail -1 gpurun_out/bench_${TAG}_g_$v.log | cut -c80-140)"
done
echo done
