set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | grep "Model name" >> gpurun_out/host.txt
timeout -k 10 300 python bench.py --arch micro --clips 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_micro.log 2>&1 || { echo "micro bench failed"; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_large.log 2>&1 || { echo "large bench failed"; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o large -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_r01.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
