#!/bin/bash
# Lanes: stagger and stream-priority A/B at 2 lanes (C3), 4 lanes once.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s11}
run() { # env lanes extra
  env $1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --lanes $2 $3 > $O/b_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/b_$TAG.json').readlines()[-1]); print('$1 lanes $2 $3', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline_encoder']['avg_launch_us'], d['gathered']['complete'])"
}
run MWX_STREAM_PRIO= 2 && run MWX_STREAM_PRIO=enc_low 2 && run MWX_STREAM_PRIO=dec_high 2 && \
run MWX_STREAM_PRIO= 2 "--lane-stagger 0.3" && run MWX_STREAM_PRIO=enc_low 2 "--lane-stagger 0.3" && \
run MWX_STREAM_PRIO= 2 && run MWX_STREAM_PRIO=enc_low 2 && run MWX_STREAM_PRIO=enc_low 3 && run MWX_STREAM_PRIO=enc_low 4
