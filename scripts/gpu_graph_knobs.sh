# decode-step graph submission knobs (HIP runtime env) on the greedy bench
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/knob.log 2>&1 || { echo "bench failed: $*"; tail -3 gpurun_out/knob.log; return 1; }
  echo "$* -> $(grep -o '"value": [0-9.]*' gpurun_out/knob.log | head -1)"
}
run X=0 && run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run DEBUG_HIP_GRAPH_BATCH_SIZE=64 && run DEBUG_HIP_GRAPH_BATCH_SIZE=1024 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=1
