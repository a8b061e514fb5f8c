#!/bin/bash
# Refactored lanes runner on the GPU: C3 default (no CPU baseline), beam-5
# 30-s leg at 2 lanes and 1 lane.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s18}
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
tail -1 $O/bench_$TAG.json | cut -c1-160
timeout -k 10 400 python -u bench.py --beam 5 --steps 4 --no-cpu-baseline > $O/bench_${TAG}_b5.json 2>> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_${TAG}_b5.json | cut -c1-160
timeout -k 10 400 python -u bench.py --beam 5 --lanes 1 --steps 2 --no-cpu-baseline > $O/bench_${TAG}_b5_1lane.json 2>> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_${TAG}_b5_1lane.json | cut -c1-160
