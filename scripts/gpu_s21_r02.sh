#!/bin/bash
# Grouped cross-attention (beam): both halves of a key batch in flight; full
# -m gpu suite, beam-5 one-lane legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s21}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 400 python -u bench.py --beam 5 --lanes 1 --steps 2 --no-cpu-baseline > $O/bench_${TAG}_b5_1lane.json 2>> $O/bench_$TAG.err || exit 3
python -c "import json; d=json.loads(open('$O/bench_${TAG}_b5_1lane.json').readlines()[-1]); print('beam5 1 lane', d['value'], d['roofline']['avg_launch_us'])"
done
timeout -k 10 400 python -u bench.py --beam 5 --steps 4 --no-cpu-baseline > $O/bench_${TAG}_b5.json 2>> $O/bench_$TAG.err || exit 3
python -c "import json; d=json.loads(open('$O/bench_${TAG}_b5.json').readlines()[-1]); print('beam5 2 lanes', d['value'], d['roofline']['avg_launch_us'])"
