#!/bin/bash
# Ping-pong encoder GEMM schedule: encoder/GEMM parity tests with it on, then
# C3 A/B on one lane (encoder GEMM time visible) and on two lanes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s15}
MWX_GEMM_PP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "encoder or v3_geometry_greedy or batch32 or base_f16 or mel" > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() { # env extra
  env $1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline $2 > $O/b_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/b_$TAG.json').readlines()[-1]); e=d['roofline_encoder'] if d.get('one_lane') is None else d['one_lane']['roofline_encoder']; print('$1 $2', d['value'], d['ms_per_step'], d['roofline_encoder']['avg_launch_us'], d['roofline_encoder']['frac'], e['frac'], d['gathered']['complete'])"
}
run MWX_GEMM_PP=1 "--lanes 1 --steps 3" && run MWX_GEMM_PP=0 "--lanes 1 --steps 3" && run MWX_GEMM_PP=1 "--lanes 1 --steps 3" && run MWX_GEMM_PP=0 "--lanes 1 --steps 3" && \
run MWX_GEMM_PP=0 "--lanes 2" && run MWX_GEMM_PP=1 "--lanes 2"
