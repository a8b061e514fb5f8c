#!/bin/bash
# A/B of the fused decode layer (gemm_ln + residual epilogues, MWX_DEC_FUSED=1)
# against the round-1 split-K + LayerNorm chain (MWX_DEC_FUSED=0): parity
# subset, then bench legs alternating, then a kernel trace of the fused build.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -q \
  --timeout 300 --timeout-method thread \
  -k "greedy or batch_equals or beam_search_replay or tiny or long_form or v3_geometry_greedy or batch32 or base_f16" \
  > gpurun_out/fused_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/fused_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for f in 1 0 1 0; do
  MWX_DEC_FUSED=$f timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_fused${f}_$RANDOM.json 2> gpurun_out/bench_err.log || exit 3
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fused" -o prof \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_fused.log" 2>&1
echo "prof rc=$?"
