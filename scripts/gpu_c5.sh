# MX-fp8 MFMA layout probe + C5-shaped bench (large-v3 bf16, beam 5, 10-min clips, 32 per GPU).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./scripts/probe/mfma_scale_probe > gpurun_out/mfma_scale_probe.txt 2>&1; echo "probe rc=$?" >> gpurun_out/mfma_scale_probe.txt
cat gpurun_out/mfma_scale_probe.txt
timeout -k 10 900 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --beam 5 --clip-seconds 600 > gpurun_out/bench_c5_bf16.log 2>&1 || { echo "c5 bench failed"; tail -20 gpurun_out/bench_c5_bf16.log; exit 1; }
tail -1 gpurun_out/bench_c5_bf16.log | cut -c1-300
