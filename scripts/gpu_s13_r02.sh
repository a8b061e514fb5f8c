#!/bin/bash
# PMC passes of the current build (one lane: per-kernel attribution without a
# concurrent batch): FETCH_SIZE, WRITE_SIZE, MFMA busy; then the beam-5 A/B of
# the grouped cross-attention's constant-count load stream.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s13}
B="python3 $GRAFT_REPO_ROOT/bench.py --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline"
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$C -o pmc -- $B > $O/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; exit 5; }
done
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${TAG}_MFMA -o pmc -- $B > $O/pmc_${TAG}_MFMA.log 2>&1 || { echo "pmc MFMA failed"; exit 5; }
cd "$GRAFT_REPO_ROOT"
python scripts/pmc_report.py $O $TAG --md $O/pmc_${TAG}.md > $O/pmc_${TAG}_report.txt 2>&1 || echo "report failed"
run() { # env extra
  env $1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline $2 > $O/b_$TAG.json 2>> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 3; }
  python -c "import json,sys; d=json.loads(open('$O/b_$TAG.json').readlines()[-1]); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['gathered']['complete'])"
}
run MWX_STREAM_PRIO=enc_low "--lanes 2" && run MWX_STREAM_PRIO=enc_low "--lanes 2 --lane-prio high,normal" && \
run MWX_STREAM_PRIO=enc_low "--lanes 2 --lane-prio high,low" && run MWX_STREAM_PRIO=both "--lanes 2" && \
run GPU_MAX_HW_QUEUES=8 "--lanes 2" && run GPU_MAX_HW_QUEUES=8 "--lanes 3" && \
run MWX_STREAM_PRIO=enc_low "--lanes 3 --lane-prio high,normal,low" && run MWX_STREAM_PRIO=enc_low "--lanes 2" && \
run MWX_XATTN_NBC=0 "--beam 5 --lanes 1 --steps 2" && run MWX_XATTN_NBC=1 "--beam 5 --lanes 1 --steps 2" && \
run MWX_XATTN_NBC=0 "--beam 5 --lanes 1 --steps 2" && run MWX_XATTN_NBC=1 "--beam 5 --lanes 1 --steps 2"
