#!/bin/bash
# Logits processing: merged workgroup reductions (fewer barriers); full -m gpu
# suite, smoke, C2 legs, default bench with CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s22}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail $O/smoke_$TAG.log; exit 2; }
tail -1 $O/smoke_$TAG.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${TAG}_c2.json 2>> $O/bench_$TAG.err || exit 3
python -c "import json; d=json.loads(open('$O/bench_${TAG}_c2.json').readlines()[-1]); print('C2', d['value'], d['ms_per_step'])"
done
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
tail -1 $O/bench_$TAG.json | cut -c1-160
