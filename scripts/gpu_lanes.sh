#!/bin/bash
# Concurrent batches (lanes) A/B: C3 bench at 1, 2, 3 lanes, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-lanes}
for ln in 1 2 3 2 1; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --lanes $ln > $O/bench_${TAG}_l$ln.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/bench_${TAG}_l$ln.json').readlines()[-1]); print('lanes $ln', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline_encoder']['avg_launch_us'], d['gathered'])"
done
