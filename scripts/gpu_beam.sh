# Beam-search (service default beam 5) and long-form bench legs + kernel profile of the beam run.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-beam}
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --clip-seconds 90 > gpurun_out/bench_${TAG}_long.log 2>&1 || { echo "long bench failed"; tail -20 gpurun_out/bench_${TAG}_long.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_long.log | cut -c1-250
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam 5 > gpurun_out/bench_${TAG}_b5.log 2>&1 || { echo "beam bench failed"; tail -20 gpurun_out/bench_${TAG}_b5.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_b5.log | cut -c1-250
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o beam -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
