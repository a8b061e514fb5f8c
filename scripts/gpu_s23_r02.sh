#!/bin/bash
# Kernel trace of the final build's default (2-lane) bench, summarised on the box.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s23}
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o greedy -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 4; }
cd "$GRAFT_REPO_ROOT"
python scripts/prof_summary.py $O/prof_$TAG/greedy_results.db $O/prof_${TAG}_kernel_stats.md > /dev/null && rm -rf $O/prof_$TAG
tail -1 $O/prof_$TAG.log | cut -c1-120
echo done
