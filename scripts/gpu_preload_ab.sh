# Kernel-argument preload A/B: libmwx.so built with -amdgpu-kernarg-preload-count=16
# against libmwx_base.so (same sources, no preload): GPU tests on the preload
# build, greedy and beam-5 legs both ways, greedy profile of the preload build.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-kpl}
L=sentiric-stt-whisper-service_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
cp $L/libmwx.so $L/libmwx_pl.so
for v in pl base pl base; do
  cp $L/libmwx_$v.so $L/libmwx.so
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_g_$v.log 2>&1 || { echo "greedy bench failed"; tail -20 gpurun_out/bench_${TAG}_g_$v.log; exit 1; }
  echo "$v greedy: $(tail -1 gpurun_out/bench_${TAG}_g_$v.log | cut -c80-140)"
done
for v in pl base; do
  cp $L/libmwx_$v.so $L/libmwx.so
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5_$v.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5_$v.log; exit 1; }
  echo "$v beam: $(tail -1 gpurun_out/bench_${TAG}_b5_$v.log | cut -c80-140)"
done
cp $L/libmwx_pl.so $L/libmwx.so
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o greedy -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
