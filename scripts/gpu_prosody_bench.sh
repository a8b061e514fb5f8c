# Prosody bench leg + its kernel profile.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-pb}
timeout -k 10 300 python bench.py --prosody --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o pros -- python3 $GRAFT_REPO_ROOT/bench.py --prosody --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; exit 1; }
echo done
