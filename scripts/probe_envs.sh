cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
P=./scripts/probe/dec_chain_probe
for cfg in "MWX_DEC_MT1=0" "MWX_SPLITK_KSMAX=4" "MWX_SPLITK_KSMAX=2" "MWX_SKINNY_NW=8" "MWX_SKINNY_NW=5" "MWX_SPLITK_KSMAX=2 MWX_DEC_MT1=0"; do
  echo "== $cfg" >> gpurun_out/r04b_probe_env.out
  env $cfg PROBE_ONLY=FULL timeout -k 5 60 $P 32 10 >> gpurun_out/r04b_probe_env.out 2>&1 || exit 1
  env $cfg PROBE_ONLY=split timeout -k 5 60 $P 32 10 >> gpurun_out/r04b_probe_env.out 2>&1 || exit 1
  env $cfg PROBE_ONLY=skinny timeout -k 5 60 $P 32 10 >> gpurun_out/r04b_probe_env.out 2>&1 || exit 1
done
