set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" "FETCH_SIZE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_xa_$i -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --decode-steps 8 --beam 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_xa_$i.log 2>&1) || { echo "pmc $i failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc_xa_$i.log; exit 1; }
done
echo ok
