# Prosody parity on the GPU (kernel vs reference golden vectors / oracle) and
# the SttEngine end-to-end test that now carries the prosody fields.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-prosody}
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_prosody.py tests/test_stt_engine.py > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "passed|failed|serial runs" gpurun_out/tests_$TAG.log | cut -c1-400
echo done
