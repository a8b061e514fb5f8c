# PMC passes over the prosody bench leg (one counter group per rocprofv3 run)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-ppmc}
i=0
for C in "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$i -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --prosody --steps 2 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$i.log 2>&1) || { echo "pmc $C failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo pmc done
