#!/bin/bash
# Cross-attention constant-batch-count load stream: parity subset, then C3
# A/B (MWX_XATTN_NBC) and the concurrent-lanes A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s10}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() { # env lanes
  env $1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --lanes $2 > $O/b_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/b_$TAG.json').readlines()[-1]); print('$1 lanes $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline_encoder']['avg_launch_us'], d['gathered']['complete'])"
}
run MWX_XATTN_NBC=0 1 && run MWX_XATTN_NBC=1 1 && run MWX_XATTN_NBC=0 1 && run MWX_XATTN_NBC=1 1 && \
run MWX_XATTN_NBC=1 2 && run MWX_XATTN_NBC=1 3 && run MWX_XATTN_NBC=1 2
