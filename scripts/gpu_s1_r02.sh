#!/bin/bash
# Round-2 re-entry check: the full -m gpu suite on the committed build, then the
# decode-chain probe (unprofiled per-launch times of the decode kernels).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > $O/tests_s1.log 2>&1
rc=$?
tail -3 $O/tests_s1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd scripts/probe && timeout -k 10 120 ./dec_chain_probe 32 10 > $O/chain_probe_s1.txt 2>&1 || exit 4
cat $O/chain_probe_s1.txt
exit $rc
