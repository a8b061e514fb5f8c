#!/bin/bash
# Live (unprofiled) per-class launch timing of the decode kernels, fused vs legacy.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cls in dec_gemm dec_attn_self dec_attn_cross; do
  for f in 1 0; do
    MWX_DEC_FUSED=$f timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      --perf-class $cls > gpurun_out/cls_${cls}_f$f.json 2> gpurun_out/cls_err.log || exit 3
  done
done
