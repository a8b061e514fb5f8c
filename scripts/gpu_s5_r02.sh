#!/bin/bash
# Full -m gpu suite on the current build (incremental log-mel, encoder
# attention, batched mel, run-ahead), C3 bench, streaming partial-latency leg
# with and without the incremental log-mel.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s5}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_$TAG.json | cut -c1-160
for v in "" "MWX_NO_MEL_CACHE=1"; do
  env $v timeout -k 10 300 python -u bench.py --stream --arch base-rich --wtype f16 --steps 2 --warmup 1 > $O/stream_$TAG.json 2>> $O/bench_$TAG.err || exit 3
  echo "stream [$v] $(tail -1 $O/stream_$TAG.json | cut -c1-400)"
done
