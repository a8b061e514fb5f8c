#!/bin/bash
# Default bench (2 lanes, 6 batches), C5 leg, kernel trace of the default bench.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s14}
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
tail -1 $O/bench_$TAG.json | cut -c1-160
timeout -k 10 600 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_${TAG}_c5.json 2>> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_${TAG}_c5.json | cut -c1-160
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o greedy -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 4; }
cd "$GRAFT_REPO_ROOT"
# (the trace database exceeds what gpurun copies back: summarise it here)
python scripts/prof_summary.py $O/prof_$TAG/greedy_results.db $O/prof_${TAG}_kernel_stats.md > /dev/null && rm -rf $O/prof_$TAG
echo done
