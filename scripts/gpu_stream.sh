set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-st}
timeout -k 10 500 python -u -m pytest tests/test_stt_stream.py tests/test_stt_engine.py -m gpu -x -v -rf --timeout 400 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tests_$TAG.log | cut -c1-200
