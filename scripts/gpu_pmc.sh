# HBM traffic of the decode kernels from PMC counters: FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes (kernel-trace only, no API traces),
# short decode (8 steps) since every dispatch gets a counter row.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-pmc}
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$C -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$C.log 2>&1) || { echo "pmc $C failed"; exit 1; }
done
echo pmc done
