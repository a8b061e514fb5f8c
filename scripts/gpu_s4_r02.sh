#!/bin/bash
# Batched log-mel + leaner encoder attention: mel / encoder / greedy parity
# subset, C3 bench, kernel trace (per-kernel stats) of one bench step.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s4}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -x -q -rf --timeout 300 --timeout-method thread \
  -k "mel or encoder or greedy or v3_geometry_greedy or batch32 or base_f16 or long_form or runahead" > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_$TAG.json | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd -d $O/prof_$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_$TAG.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python3 scripts/prof_summary.py $(find $O/prof_$TAG -name '*.db' | head -1) $O/kstats_$TAG.md > /dev/null 2>&1; head -24 $O/kstats_$TAG.md
