#!/bin/bash
# fp8 (MWX_COMPUTE_MXFP8) decoder weights + fp8 cross K/V cache: parity, then
# bench legs (bf16 greedy default, fp8 greedy, C5-shaped fp8 beam-5 600 s)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -v \
  --timeout 400 --timeout-method thread -k "mx or fp8 or greedy_matches or batch_equals" \
  > gpurun_out/fp8_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/fp8_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_bf16.json 2>gpurun_out/b_err.log || exit 3
timeout -k 10 300 python -u bench.py --fp8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_fp8.json 2>>gpurun_out/b_err.log || exit 3
timeout -k 10 400 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b_c5.json 2>>gpurun_out/b_err.log || exit 3
