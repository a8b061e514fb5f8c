#!/bin/bash
# prefill-vs-stepwise isolation: the teacher-forced logits test under knobs
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T="tests/test_gpu_prefill.py -k logits_equal"
for cfg in "" "MWX_PREFILL_XNQ=1" "MWX_PREFILL_SPAN=1" "MWX_PREFILL_SPAN=1 MWX_PREFILL_XNQ=1"; do
  env $cfg timeout -k 10 300 python -u -m pytest $T -v -rf --timeout 250 --timeout-method thread > gpurun_out/d2.out 2>&1; rc=$?
  echo "== [$cfg] rc=$rc"; grep -E "PASSED|FAILED|AssertionError: \(" gpurun_out/d2.out | head -8
  [ $rc -ge 124 ] && exit $rc
done
exit 0
