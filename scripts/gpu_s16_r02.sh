#!/bin/bash
# Round-2 closing evidence: full -m gpu suite, smoke, default bench (2 lanes,
# CPU baseline), one-lane C3 and C2 legs, kernel traces (summarised on the box).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s16}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail $O/smoke_$TAG.log; exit 2; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
tail -1 $O/bench_$TAG.json | cut -c1-160
timeout -k 10 300 python -u bench.py --lanes 1 --steps 3 --no-cpu-baseline > $O/bench_${TAG}_1lane.json 2>> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_${TAG}_1lane.json | cut -c1-160
timeout -k 10 300 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${TAG}_c2.json 2>> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_${TAG}_c2.json | cut -c1-160
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_${TAG}_1lane -o greedy -- python3 $GRAFT_REPO_ROOT/bench.py --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_${TAG}_1lane.log 2>&1 || { echo "prof failed"; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${TAG}_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_${TAG}_c2.log 2>&1 || { echo "c2 prof failed"; exit 4; }
cd "$GRAFT_REPO_ROOT"
python scripts/prof_summary.py $O/prof_${TAG}_1lane/greedy_results.db $O/prof_${TAG}_1lane_kernel_stats.md > /dev/null && rm -rf $O/prof_${TAG}_1lane
python scripts/prof_summary.py $O/prof_${TAG}_c2/c2_results.db $O/prof_${TAG}_c2_kernel_stats.md > /dev/null && rm -rf $O/prof_${TAG}_c2
echo done
