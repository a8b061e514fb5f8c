#!/bin/bash
# Cross-attention: two key batches and the bias requested in the prologue
# (NBC path): full -m gpu suite, then C3 one-lane A/B against the runtime-count
# kernel (MWX_XATTN_NBC=0) and the default 2-lane bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s19}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() { # env extra
  env $1 timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $2 > $O/b_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/b_$TAG.json').readlines()[-1]); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['gathered']['complete'])"
}
run MWX_XATTN_NBC=0 "--lanes 1 --steps 3" && run MWX_XATTN_NBC=1 "--lanes 1 --steps 3" && run MWX_XATTN_NBC=0 "--lanes 1 --steps 3" && run MWX_XATTN_NBC=1 "--lanes 1 --steps 3" && \
run MWX_XATTN_NBC=0 "--steps 6" && run MWX_XATTN_NBC=1 "--steps 6"
