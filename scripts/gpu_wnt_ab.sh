#!/bin/bash
# A/B: decode GEMM weight loads with the non-temporal policy (MWX_DEC_WNT) x
# 16- / 32-row blocks (MWX_DEC_MT1): chain probe (full layer) and the C3 bench.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for v in "MWX_DEC_WNT=0 MWX_DEC_MT1=1" "MWX_DEC_WNT=1 MWX_DEC_MT1=1" "MWX_DEC_WNT=0 MWX_DEC_MT1=0" "MWX_DEC_WNT=1 MWX_DEC_MT1=0"; do
  echo "[$v]"
  (cd scripts/probe && env $v PROBE_ONLY="FULL layer (" timeout -k 10 60 ./dec_chain_probe 32 10 | tail -1) || exit 4
done
for v in "MWX_DEC_WNT=0" "MWX_DEC_WNT=1" "MWX_DEC_WNT=1 MWX_DEC_MT1=0" "MWX_DEC_WNT=0"; do
  env $v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_wnt.json 2>>$O/bench_wnt.err || exit 3
  echo "C3 [$v] $(tail -1 $O/bench_wnt.json | cut -c90-140)"
done
