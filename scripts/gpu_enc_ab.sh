# encoder GEMM A/B: two libmwx.so builds swapped in place
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-enc}
for v in a b; do
  cp sentiric-stt-whisper-service_amd/libmwx_$v.so sentiric-stt-whisper-service_amd/libmwx.so
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --perf-class enc_gemm > gpurun_out/bench_${TAG}_$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_${TAG}_$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_${TAG}_$v.log | head -1) $(grep -o '"achieved": [0-9.]*' gpurun_out/bench_${TAG}_$v.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench_${TAG}_$v.log)"
done
