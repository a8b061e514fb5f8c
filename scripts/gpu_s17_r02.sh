#!/bin/bash
# Deep K/V stream for small cross-attention grids (C2, one request): full
# -m gpu suite (micro / base single-request tests run it), C2 A/B, C3 check.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s17}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() { # env extra
  env $1 timeout -k 10 300 python -u bench.py --warmup 2 --no-cpu-baseline $2 > $O/b_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/b_$TAG.json').readlines()[-1]); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['gathered']['complete'])"
}
C2="--arch base --wtype f16 --clips 1 --lanes 1 --steps 10"
run MWX_XATTN_DEEP=0 "$C2" && run MWX_XATTN_DEEP=1 "$C2" && run MWX_XATTN_DEEP=0 "$C2" && run MWX_XATTN_DEEP=1 "$C2" && \
run MWX_XATTN_DEEP=1 "--steps 6"
