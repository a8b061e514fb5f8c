#!/bin/bash
# DPP wave reductions (LayerNorm, attention softmax, logits max) + early value
# loads in the greedy self-attention: chain probe, full -m gpu suite, C3 bench.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-s8}
for v in "MWX_SELF_EARLYV=0" "MWX_SELF_EARLYV=1"; do
  echo "[$v]"
  (cd scripts/probe && for op in ln_dec "self_attn" "cross_attn" "FULL layer ("; do env $v PROBE_ONLY="$op" timeout -k 10 60 ./dec_chain_probe 32 10 | tail -1 || exit 4; done) || exit 4
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1
rc=$?
tail -3 $O/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in "MWX_SELF_EARLYV=1" "MWX_SELF_EARLYV=0" "MWX_SELF_EARLYV=1"; do
  env $v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$TAG.json 2>> $O/bench_$TAG.err || exit 3
  echo "C3 [$v] $(tail -1 $O/bench_$TAG.json | cut -c90-140)"
done
