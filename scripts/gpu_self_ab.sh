# self-attention A/B: new wave-per-head kernel vs the workgroup-per-head one
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-sab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for v in new old; do
  if [ $v = old ]; then export MWX_SELF_ATTN_WG=1; fi
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --perf-class dec_attn_self > gpurun_out/bench_${TAG}_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_${TAG}_$v.log; exit 1; }
  echo "$v greedy $(grep -o '"value": [0-9.]*' gpurun_out/bench_${TAG}_$v.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench_${TAG}_$v.log)"
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 --perf-class dec_attn_self > gpurun_out/bench_${TAG}_${v}_b5.log 2>&1 || { echo "beam bench failed"; exit 1; }
  echo "$v beam5 $(grep -o '"value": [0-9.]*' gpurun_out/bench_${TAG}_${v}_b5.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench_${TAG}_${v}_b5.log)"
done
