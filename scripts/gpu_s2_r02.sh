#!/bin/bash
# Stream-pattern probe (cross-attention bytes), decode-chain probe on the
# current build, default bench, and a kernel trace (rocpd db) of a short
# decode for the inter-step gaps.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s2}
(cd scripts/probe && timeout -k 10 120 ./stream_probe 32 > $O/stream_probe_$TAG.txt 2>&1) || exit 4
cat $O/stream_probe_$TAG.txt
(cd scripts/probe && PROBE_ONLY=ln_dec timeout -k 10 120 ./dec_chain_probe 32 10 > $O/chain_probe_$TAG.txt 2>&1) || exit 4
cat $O/chain_probe_$TAG.txt
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit 3
tail -1 $O/bench_$TAG.json | cut -c1-220
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f rocpd -d $O/prof_$TAG -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --decode-steps 40 --no-cpu-baseline > $O/prof_$TAG.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && DB=$(find $O/prof_$TAG -name '*.db' | head -1) && python3 scripts/prof_gaps.py "$DB" 1 > $O/gaps_$TAG.md 2>&1
cat $O/gaps_$TAG.md | head -40
