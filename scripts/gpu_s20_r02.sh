#!/bin/bash
# Grouped cross-attention bias-with-slabs: beam / best-of parity tests, beam-5
# A/B-free check (one lane and two lanes), default bench with CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s20}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail $O/smoke_$TAG.log; exit 2; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 400 python -u bench.py --beam 5 --lanes 1 --steps 2 --no-cpu-baseline > $O/bench_${TAG}_b5_1lane.json 2>> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_${TAG}_b5_1lane.json | cut -c1-120
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
tail -1 $O/bench_$TAG.json | cut -c1-160
