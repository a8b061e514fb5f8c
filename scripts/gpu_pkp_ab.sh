# Packed-P cross-attention A/B (MWX_XATTN_PKP=1; bit-exact by construction) with the
# UB=4 self-attention default: full GPU tests with PKP on, greedy and beam-5 legs
# both ways, beam and greedy profiles with PKP on.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-pab}
MWX_XATTN_PKP=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for v in 0 1; do
  MWX_XATTN_PKP=$v timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5_p$v.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5_p$v.log; exit 1; }
  echo "pkp$v beam: $(tail -1 gpurun_out/bench_${TAG}_b5_p$v.log | cut -c80-140)"
  MWX_XATTN_PKP=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_g_p$v.log 2>&1 || { echo "greedy bench failed"; exit 1; }
  echo "pkp$v greedy: $(tail -1 gpurun_out/bench_${TAG}_g_p$v.log | cut -c80-140)"
done
cd /tmp && MWX_XATTN_PKP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_b5 -o beam -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_b5.log 2>&1 || { echo "prof failed"; exit 1; }
MWX_XATTN_PKP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_g -o greedy -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_g.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
