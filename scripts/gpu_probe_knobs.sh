#!/bin/bash
# decode GEMM knob sweep on the chain probe (unprofiled, in-graph)
cd "$GRAFT_REPO_ROOT" || exit 1
P=scripts/probe/dec_chain_probe
o=gpurun_out/probe_knobs.txt
: > $o
for nw in 16 10 8 5 4; do
  echo "== MWX_SKINNY_NW=$nw" >> $o
  PROBE_ONLY=skinny_fc1 MWX_SKINNY_NW=$nw timeout -k 10 60 $P 32 10 >> $o 2>&1 || exit 3
done
for ks in 8 5 4 2; do
  echo "== MWX_SPLITK_KSMAX=$ks" >> $o
  PROBE_ONLY=splitk MWX_SPLITK_KSMAX=$ks timeout -k 10 60 $P 32 10 >> $o 2>&1 || exit 3
done
echo "== default, full" >> $o
timeout -k 10 150 $P 32 10 >> $o 2>&1
