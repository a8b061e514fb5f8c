#!/bin/bash
# Round-2 evidence: default bench (C3 greedy) + its kernel trace, C2 leg
# (base f16, 1 clip) + trace, C5 leg (MX-fp8 beam 5, 600-s clips), PMC passes
# (FETCH_SIZE, WRITE_SIZE, MFMA busy) on a short decode, each in its own run.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
TAG=${1:-r02}
B="python3 $GRAFT_REPO_ROOT/bench.py"
timeout -s KILL 60 rocprofv3 -L > $O/${TAG}_counters_list.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_bench.json 2>$O/${TAG}_err.log || { echo "bench failed"; exit 3; }
tail -1 $O/${TAG}_bench.json | cut -c1-160
timeout -k 10 300 python -u bench.py --arch base --wtype f16 --clips 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench_c2.json 2>>$O/${TAG}_err.log || { echo "c2 bench failed"; exit 3; }
tail -1 $O/${TAG}_bench_c2.json | cut -c1-160
timeout -k 10 500 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --steps 1 --warmup 1 --no-cpu-baseline > $O/${TAG}_bench_c5.json 2>>$O/${TAG}_err.log || { echo "c5 bench failed"; exit 3; }
tail -1 $O/${TAG}_bench_c5.json | cut -c1-160
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_greedy -o greedy -- $B --steps 1 --warmup 1 --no-cpu-baseline > $O/${TAG}_prof_greedy.log 2>&1 || { echo "prof failed"; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_c2 -o c2 -- $B --arch base --wtype f16 --clips 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_prof_c2.log 2>&1 || { echo "c2 prof failed"; exit 4; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$C -o pmc -- $B --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline > $O/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; exit 5; }
done
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${TAG}_MFMA -o pmc -- $B --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline > $O/pmc_${TAG}_MFMA.log 2>&1 || { echo "pmc MFMA failed"; exit 5; }
echo evidence done
