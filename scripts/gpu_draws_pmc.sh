set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
(cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_draws -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/draws_timing.py > $GRAFT_REPO_ROOT/gpurun_out/pmc_draws.log 2>&1) || { echo "pmc failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_draws.log; exit 1; }
echo ok
