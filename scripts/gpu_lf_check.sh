# long-form parity test under the self-attention / packed-P variants
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "MWX_SELF_UB=8 MWX_XATTN_PKP=0" "MWX_SELF_UB=8 MWX_XATTN_PKP=1" "MWX_SELF_UB=4 MWX_XATTN_PKP=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 200 --timeout-method thread -k "long_form or rich or beam" > gpurun_out/lf.log 2>&1; rc=$?
  echo "$cfg: rc=$rc $(tail -1 gpurun_out/lf.log)"
  [ $rc -le 1 ] || exit 1
done
