# Cross-attention rows-per-batch sweep (MWX_XUB = 8, 12, 16): greedy bench legs.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for U in 8 12 16; do
  MWX_XUB=$U timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_xub$U.log 2>&1 || { echo "bench $U failed"; tail -5 gpurun_out/bench_xub$U.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_xub$U.log').read().strip().splitlines()[-1]); print($U, d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
