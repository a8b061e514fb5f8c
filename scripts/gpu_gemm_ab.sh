# Encoder GEMM A/B: kernel-trace profiles of an encoder-dominated run (8 decode steps)
# with and without the XCD tile remap, bf16 and MX-fp8; then quick parity tests.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-gab}
timeout -k 10 300 python -u -m pytest tests -m gpu -k "encoder or mx or greedy" -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
cd /tmp
for V in remap noremap; do
  for F in "" "--fp8"; do
    N=${V}${F:+_fp8}
    if [ $V = noremap ]; then export MWX_NO_XCD_REMAP=1; else unset MWX_NO_XCD_REMAP; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$N -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --decode-steps 8 $F > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$N.log 2>&1 || { echo "prof $N failed"; exit 1; }
  done
done
echo done
