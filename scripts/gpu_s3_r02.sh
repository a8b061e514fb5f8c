#!/bin/bash
# Run-ahead greedy decode + non-temporal cross K/V loads: full -m gpu suite,
# then A/B bench legs (C3 greedy: default / MWX_XATTN_NT=0 / MWX_NO_RUNAHEAD=1;
# C2 base f16 B=1: default / MWX_NO_RUNAHEAD=1).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > $O/tests_$TAG.log 2>&1
rc=$?
tail -5 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
B="python -u bench.py --no-cpu-baseline"
for v in "" "MWX_XATTN_NT=0" "MWX_NO_RUNAHEAD=1" ""; do
  env $v timeout -k 10 300 $B --steps 3 --warmup 1 > $O/bench_${TAG}_c3.json 2>>$O/bench_$TAG.err || exit 3
  echo "C3 [$v] $(tail -1 $O/bench_${TAG}_c3.json | cut -c90-170)"
done
for v in "" "MWX_NO_RUNAHEAD=1" ""; do
  env $v timeout -k 10 300 $B --arch base --wtype f16 --clips 1 --steps 10 --warmup 2 > $O/bench_${TAG}_c2.json 2>>$O/bench_$TAG.err || exit 3
  echo "C2 [$v] $(tail -1 $O/bench_${TAG}_c2.json | cut -c90-170)"
done
