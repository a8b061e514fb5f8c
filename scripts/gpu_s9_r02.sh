#!/bin/bash
# Fresh-container state check: full -m gpu suite, default bench (with the CPU
# baseline), kernel trace of the benched build.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s9}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_$TAG.json | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o greedy -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 4; }
echo done
