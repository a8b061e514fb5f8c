#!/bin/bash
# One parameterised GPU run recipe (gpurun). Usage, on the box:
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
# steps (each under its own time limit; the first failure ends the run):
#   tests      pytest -m gpu (one process)
#   smoke      __graft_entry__.smoke()
#   abh / ab<commit>  2-lane bench of HEAD's / an older build's library (ablib/, built beforehand)
#   bench      default bench line (C3: 2 lanes + one-lane value + CPU baseline)
#   benchq     default bench without the CPU baseline (quick)
#   bench1     C3 on one lane
#   c2         C2: base f16, one clip per request
#   c2nt       C2 with the cross K/V streamed non-temporally (A/B of the MALL-resident default)
#   b5one      beam 5 on one lane (b5onenog: decoder groups' f16 cross-attention on v_dot2)
#   stream / streamr / streamv3r  streaming partial latency: base (220-token windows + fallbacks),
#              base-rich (EOT / timestamps, r02's workload), large-v3-rich
#   bench1nts / benchqnts  C3 one lane / 2 lanes with token_timestamps off (A/B of the round-3 regression)
#   probe      the decode-chain probe (scripts/probe/dec_chain_probe): fused seams bit-exact + per-layer times
#   mfstest    the MX-fp8 tests with the MFMA-score cross-attention (MWX_XATTN_MFS=1)
#   c5mfs / c5one  C5 on one lane with / without the MFMA scores
#   bench1np / bench1g0  one lane without the prompt prefill / with row-major encoder tile order
#   bench1g16 / bench1g32 / pmcg32  encoder tile-order group of 16 / 32 row tiles (one lane; FETCH pass)
#   benchqnp / bench1np8  the instrumented (span) step graph replayed only once (A/B of the live timing's cost)
#   b5         beam 5 (service default decode), C3 shape
#   c5         C5: MX-fp8, beam 5, 600-s long-form clips
#   prompt     long-form leg with previous-window text carried as the prompt
#   prof       rocprofv3 --kernel-trace --stats of the exact default bench command
#   prof1      the same for --lanes 1
#   profc2     kernel trace of the C2 leg
#   profb5     kernel trace of beam 5 (one lane)
#   profc5     kernel trace of the C5 leg (one lane, one 600-s batch)
#   profsvc    kernel trace of one service-default batch (one lane)
#   pmcb5      instruction-mix / stall counters of a short beam-5 decode, bf16 and MX-fp8
#   pmc        FETCH_SIZE / WRITE_SIZE / MFMA-busy passes (each its own run) on a short decode
# Outputs go to gpurun_out/<TAG>_*; copy the summaries to be judged into profiles/.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$O"
TAG=$1
shift
B="python3 $GRAFT_REPO_ROOT/bench.py"
run() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$secs" "$@" > "$O/${TAG}_${name}.out" 2> "$O/${TAG}_${name}.err"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "$name failed rc=$rc"
    tail -n 30 "$O/${TAG}_${name}.out" "$O/${TAG}_${name}.err"
    exit $rc
  fi
  tail -1 "$O/${TAG}_${name}.out" | cut -c1-400
}
for s in "$@"; do
  case $s in
    c5pad) run c5pad 700 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/pad/libmwx.so python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    c5h) run c5h 700 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/libmwx_head.so python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    b5h) run b5h 500 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/libmwx_head.so python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    b5e_*)  # beam 5 on one lane with one engine knob: b5e_<VAR>_<value> (MWX_<VAR>=<value>)
      kv=${s#b5e_}; var=MWX_${kv%_*}; val=${kv##*_}
      run "$s" 500 env "$var=$val" python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    b1e_*)  # C3 on one lane with one engine knob: b1e_<VAR>_<value> (MWX_<VAR>=<value>)
      kv=${s#b1e_}; var=MWX_${kv%_*}; val=${kv##*_}
      run "$s" 400 env "$var=$val" python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    c5e_*)  # C5 on one lane with one engine knob: c5e_<VAR>_<value> (MWX_<VAR>=<value>)
      kv=${s#c5e_}; var=MWX_${kv%_*}; val=${kv##*_}
      run "$s" 700 env "$var=$val" python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    sharedgreedy) run sharedgreedy 600 env MWX_DEC_SHARED_MIN=17 python -u -m pytest tests/test_gpu_shapes.py -k "batch32_equals_single or row_block" -m gpu -v -s -rf --timeout 500 --timeout-method thread ;;
    sharedkh2) run sharedkh2 600 env MWX_DEC_SHARED_KH=2 python -u -m pytest tests/test_gpu_shapes.py -k "row_block or beam_batch" -m gpu -v -s -rf --timeout 500 --timeout-method thread ;;
    probekh) for v in 1 2; do for k in logits skinny_fc1; do run "probekh_${v}_$k" 200 env MWX_DEC_SHARED_KH=$v PROBE_ONLY="$k" ./scripts/probe/dec_chain_probe 160 10 || exit 6; done; done ;;
    sharedtests) run sharedtests 900 python -u -m pytest tests/test_gpu_shapes.py -k "row_block or beam_batch or group_of_7" -m gpu -v -s -rf --timeout 600 --timeout-method thread ;;
    abb*)  # the same for beam 5 (ablib/libmwx_<build>.so, 2 lanes)
      v=${s#abb}; [ "$v" = h ] && v=head
      run "${s}_$(date +%s)" 500 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/libmwx_$v.so python -u bench.py --beam 5 --steps 4 --warmup 1 --no-cpu-baseline --no-one-lane ;;
    ab*)  # A/B of builds on one box: ablib/libmwx_<build>.so, 2 lanes
      v=${s#ab}; [ "$v" = h ] && v=head
      run "${s}_$(date +%s)" 400 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/libmwx_$v.so python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-one-lane ;;
    svc) run svc 700 python -u bench.py --service-defaults --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    svc2) run svc2 900 python -u bench.py --service-defaults --steps 4 --warmup 1 --no-cpu-baseline --no-one-lane ;;
    fdl) run fdl 600 python -u -m pytest tests/test_gpu_fulldepth.py -k "language_auto" -m gpu -v -s -rf --durations=0 --timeout 500 --timeout-method thread ;;
    beamorcr) run beamorcr 600 python -u -m pytest tests/test_gpu_beam_oracle.py -k "not full_depth" -m gpu -v -s -rf --timeout 500 --timeout-method thread ;;
    beamorcf) run beamorcf 1000 python -u -m pytest tests/test_gpu_beam_oracle.py -k "full_depth" -m gpu -v -s -rf --durations=0 --timeout 900 --timeout-method thread ;;
    ratests) run ratests 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -k "runahead or beam or fallback or temperature or service or group_of_7 or sampl" -m gpu -v -s -rf --durations=0 --timeout 300 --timeout-method thread ;;
    ladderdiag) run ladderdiag 400 python -u scripts/probe/ladder_diag.py ;;
    laddertests) run laddertests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_beam_oracle.py -k "ladder or runahead" -m gpu -v -s -rf --durations=0 --timeout 300 --timeout-method thread ;;
    foldtests) run foldtests 600 python -u -m pytest tests/test_gpu_parity.py -k "ln_fold or rich or replay or runahead or decoder_logits or greedy" -m gpu -v -s -rf --durations=0 --timeout 300 --timeout-method thread ;;
    c2nf*) run "$s" 300 env MWX_LN_FOLD=0 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    c2f*) run "$s" 300 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    streamrnf) run streamrnf 300 env MWX_LN_FOLD=0 python -u bench.py --stream --rich --arch base --wtype f16 --steps 3 --warmup 1 ;;
    ramm) run ramm 400 python -u -m pytest tests/test_gpu_parity.py -k "runahead_mismatch or ln_fold" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    mrdiag) run mrdiag 500 python -u scripts/probe/multirank_diag.py ;;
    mrtests) run mrtests 600 python -u -m pytest tests/test_multi_rank.py -m gpu -v -s -rf --timeout 500 --timeout-method thread ;;
    newtests) run newtests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -k "extreme_scales or widening or runahead_mismatch or grouped_self or beam_search" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    pmcbs)  # beam 5 bf16 at the benched 220 steps: FETCH and LDS / MFMA passes (the self-attention's history reads)
      for x in "fetch:FETCH_SIZE" "lds:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
        n=${x%%:*}; c=${x#*:}
        (cd /tmp && run pmcbs_$n 400 rocprofv3 --pmc $c --output-format csv -d "$O/${TAG}_pmcbs_$n" -o pmc -- $B --beam 5 --lanes 1 --steps 1 --warmup 0 --no-cpu-baseline) || exit 5
        python3 scripts/pmc_mix.py "$O/${TAG}_pmcbs_$n" 14 > "$O/${TAG}_pmcbs_$n.md" || exit 5
        rm -rf "$O/${TAG}_pmcbs_$n"  # (raw CSVs exceed what gpurun copies back)
      done ;;
    c5layer) run c5layer 600 python -u -m pytest tests/test_gpu_c5.py -k "per_layer" -m gpu -v -s -rf --durations=0 --timeout 500 --timeout-method thread ;;
    pmcl)  # greedy one lane, short decode: LDS conflicts / MFMA busy of the encoder GEMMs and attention
      (cd /tmp && run pmcl 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$O/${TAG}_pmcl" -o pmc -- $B --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
      python3 scripts/pmc_mix.py "$O/${TAG}_pmcl" 14 > "$O/${TAG}_pmcl.md" || exit 5 ;;
    enctests) run enctests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fulldepth.py tests/test_gpu_shapes.py -k "encoder or greedy or mel or batch32 or fulldepth or full_depth_large_v3_greedy" -m gpu -v -s -rf --durations=0 --timeout 500 --timeout-method thread ;;
    pmcxc5)  # the MX-fp8 grouped cross-attention (C5): LDS / MFMA and FETCH passes
      (cd /tmp && run pmcxc5_lds 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$O/${TAG}_pmcxc5_lds" -o pmc -- $B --fp8 --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
      python3 scripts/pmc_mix.py "$O/${TAG}_pmcxc5_lds" 12 > "$O/${TAG}_pmcxc5_lds.md" || exit 5
      rm -rf "$O/${TAG}_pmcxc5_lds" ;;
    barprobe) run barprobe 120 ./scripts/probe/xcd_barrier_probe 4000 ;;
    tests) run tests 1150 python -u -m pytest tests -m gpu -v -s -rf --durations=0 --timeout 600 --timeout-method thread ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py --steps 20 --warmup 5 ;;
    benchq) run benchq 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline ;;
    bench1) run bench1 400 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    c2) run c2 300 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    c2nt) run c2nt 300 env MWX_XATTN_NT=1 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    mfstest) run mfstest 600 env MWX_XATTN_MFS=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -k "mxfp8" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    c5mfs) run c5mfs 700 env MWX_XATTN_MFS=1 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    c5onevd1) run c5onevd1 700 env MWX_XATTN_VD=1 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    vdtests) run vdtests 400 python -u -m pytest tests/test_gpu_parity.py -k "v_depth or mx_cross or mxfp8" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    torchgemm) run torchgemm 300 python -u scripts/probe/enc_gemm_torch.py ;;
    c5onevb4) run c5onevb4 700 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/libmwx_vb4.so python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    c5onevb1) run c5onevb1 700 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/libmwx_vb1.so python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    c5one) run c5one 700 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    bench1np) run bench1np 400 env MWX_PREFILL_MIN=0 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    bench1g0) run bench1g0 400 env MWX_GEMM_GROUP=0 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    beamtests) run beamtests 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_prefill.py -k "beam" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    b5onenra) run b5onenra 500 env MWX_NO_RUNAHEAD=1 python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    beamra) run beamra 400 python -u -m pytest tests/test_gpu_parity.py -k "runahead or beam" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    tsfull) run tsfull 600 python -u -m pytest tests/test_gpu_fulldepth.py -k "bench_workload" -m gpu -v -s -rf --timeout 600 --timeout-method thread ;;
    bench3l) run bench3l 600 python -u bench.py --lanes 3 --steps 9 --warmup 3 --no-cpu-baseline --no-one-lane ;;
    beamorc) run beamorc 900 python -u -m pytest tests/test_gpu_beam_oracle.py -m gpu -v -s -rf --timeout 800 --timeout-method thread ;;
    c5tests) run c5tests 1100 python -u -m pytest tests/test_gpu_c5.py -m gpu -v -s -rf --timeout 1000 --timeout-method thread ;;
    probe160) for k in self_attn skinny_fc1 splitk_ ln_dec; do run "probe160_$k" 200 env PROBE_ONLY="$k" ./scripts/probe/dec_chain_probe 160 10 || exit 6; done ;;
    probe160s) for v in 1 0; do for k in logits skinny_fc1 splitk_; do run "probe160s_${v}_$k" 200 env MWX_DEC_SHARED=$v PROBE_ONLY="$k" ./scripts/probe/dec_chain_probe 160 10 || exit 6; done; done ;;
    probewb) for k in logits skinny_fc1 splitk_; do run "probewb_$k" 200 env LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/ablib/wball PROBE_ONLY="$k" ./scripts/probe/dec_chain_probe 160 10 || exit 6; done ;;
    b5w) run b5w 500 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/wball/libmwx.so python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    c5w) run c5w 700 env MWX_LIB=$GRAFT_REPO_ROOT/ablib/wball/libmwx.so python -u bench.py --fp8 --beam 5 --clip-seconds 600 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline ;;
    probehalf) for v in 1 0; do for k in logits skinny_fc1; do run "probehalf_${v}_$k" 200 env MWX_DEC_SHARED_HALF=$v PROBE_ONLY="$k" ./scripts/probe/dec_chain_probe 160 10 || exit 6; done; done ;;
    probelaunch) for k in launch "empty 512" res_ splitk skinny ln_dec; do run "probe_$(echo $k | tr -d ' ')" 200 env PROBE_ONLY="$k" ./scripts/probe/dec_chain_probe 32 10 || exit 6; done ;;
    stream) run stream 300 python -u bench.py --stream --arch base --wtype f16 --steps 3 --warmup 1 ;;
    streamr) run streamr 300 python -u bench.py --stream --rich --arch base --wtype f16 --steps 3 --warmup 1 ;;
    streamv3r) run streamv3r 500 python -u bench.py --stream --rich --arch large-v3 --wtype bf16 --steps 1 --warmup 1 ;;
    streamv3) run streamv3 400 python -u bench.py --stream --arch large-v3 --wtype bf16 --steps 2 --warmup 1 ;;
    g8tests) run g8tests 300 python -u -m pytest tests/test_gpu_parity.py -k "8phase or gemm_gelu or encoder_and_cross or mx_gemm or mxfp8_encoder" -m gpu -v -s -rf --timeout 120 --timeout-method thread ;;
    bench1g8) run bench1g8 400 env MWX_GEMM_8PH=1 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    ptests) run ptests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    tr8) run tr8 120 ./scripts/probe/tr8_probe ;;
    tr16) run tr16 120 ./scripts/probe/tr16_probe ;;
    mxtests) run mxtests 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_prefill.py -k "mx or fp8" -m gpu -v -s -rf --timeout 300 --timeout-method thread ;;
    b5onenw4) run b5onenw4 500 env MWX_SELF_NW=4 python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    bench1nw4) run bench1nw4 400 env MWX_SELF_NW=4 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    c2nw4) run c2nw4 300 env MWX_SELF_NW=4 python -u bench.py --arch base --wtype f16 --clips 1 --lanes 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    b5onenog) run b5onenog 500 env MWX_XATTN_GMFMA=0 python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    b5one) run b5one 500 python -u bench.py --beam 5 --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    bench1g16) run bench1g16 400 env MWX_GEMM_GROUP=16 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    bench1g32) run bench1g32 400 env MWX_GEMM_GROUP=32 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    pmcg32) (export MWX_GEMM_GROUP=32; cd /tmp && run pmcg32_FETCH_SIZE 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/${TAG}_pmcg32_FETCH_SIZE" -o pmc -- $B --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5 ;;
    bench1nts) run bench1nts 400 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline --no-token-timestamps ;;
    benchqnts) run benchqnts 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-token-timestamps ;;
    probe) run probe 200 env PROBE_ONLY=seam ./scripts/probe/dec_chain_probe 32 10 && run probel 200 env PROBE_ONLY=layer ./scripts/probe/dec_chain_probe 32 10 ;;
    benchqnp) run benchqnp 400 env MWX_PERF_PERIOD=1000000 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline ;;
    bench1np8) run bench1np8 400 env MWX_PERF_PERIOD=1000000 python -u bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline ;;
    b5) run b5 500 python -u bench.py --beam 5 --steps 4 --warmup 1 --no-cpu-baseline ;;
    c5) run c5 700 python -u bench.py --fp8 --beam 5 --clip-seconds 600 --steps 2 --warmup 1 --no-cpu-baseline ;;
    prompt) run prompt 700 python -u bench.py --prompt-leg --steps 2 --warmup 1 --no-cpu-baseline ;;
    prof) (cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof" -o prof -- $B --steps 4 --warmup 2 --no-cpu-baseline --no-one-lane) || exit 4; python3 scripts/prof_box.py "$O/${TAG}_prof" || exit 4 ;;
    prof1) (cd /tmp && run prof1 600 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof1" -o prof -- $B --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline) || exit 4; python3 scripts/prof_box.py "$O/${TAG}_prof1" || exit 4 ;;
    profc2) (cd /tmp && run profc2 400 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_profc2" -o prof -- $B --arch base --wtype f16 --clips 1 --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline) || exit 4; python3 scripts/prof_box.py "$O/${TAG}_profc2" || exit 4 ;;
    profb5) (cd /tmp && run profb5 600 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_profb5" -o prof -- $B --beam 5 --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline) || exit 4; python3 scripts/prof_box.py "$O/${TAG}_profb5" || exit 4 ;;
    profsvc) (cd /tmp && run profsvc 600 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_profsvc" -o prof -- $B --service-defaults --lanes 1 --steps 1 --warmup 0 --no-cpu-baseline) || exit 4; python3 scripts/prof_box.py "$O/${TAG}_profsvc" || exit 4 ;;
    profc5) (cd /tmp && run profc5 700 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_profc5" -o prof -- $B --fp8 --beam 5 --clip-seconds 60 --lanes 1 --steps 1 --warmup 0 --no-cpu-baseline) || exit 4; python3 scripts/prof_box.py "$O/${TAG}_profc5" || exit 4 ;;
    pmcb5)  # instruction mix / stall counters of the beam-5 (and fp8) kernels
      (cd /tmp && run pmcb5 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$O/${TAG}_pmcb5" -o pmc -- $B --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
      (cd /tmp && run pmcc5 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$O/${TAG}_pmcc5" -o pmc -- $B --fp8 --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5 ;;
    pmcb)  # beam 5 bf16 only: mix, LDS / MFMA, fetch (the 160-row decode chain)
      for x in "mix:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "lds:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "fetch:FETCH_SIZE"; do
        n=${x%%:*}; c=${x#*:}
        (cd /tmp && run pmcb_$n 400 rocprofv3 --pmc $c --output-format csv -d "$O/${TAG}_pmcb_$n" -o pmc -- $B --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 24 --no-cpu-baseline) || exit 5
        python3 scripts/pmc_mix.py "$O/${TAG}_pmcb_$n" 14 > "$O/${TAG}_pmcb_$n.md" || exit 5
      done ;;
    pmcx)  # the grouped cross-attentions (beam 5 bf16, C5 MX-fp8): mix, LDS / MFMA / occupancy, FETCH
      for leg in b5 c5; do
        F=""; [ $leg = c5 ] && F="--fp8"
        (cd /tmp && run pmcx_${leg}_mix 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$O/${TAG}_pmcx_${leg}_mix" -o pmc -- $B $F --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
        (cd /tmp && run pmcx_${leg}_lds 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$O/${TAG}_pmcx_${leg}_lds" -o pmc -- $B $F --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
        (cd /tmp && run pmcx_${leg}_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/${TAG}_pmcx_${leg}_fetch" -o pmc -- $B $F --beam 5 --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
        for x in mix lds fetch; do python3 scripts/pmc_mix.py "$O/${TAG}_pmcx_${leg}_$x" 12 > "$O/${TAG}_pmcx_${leg}_$x.md" || exit 5; done
      done ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && run pmc_$C 400 rocprofv3 --pmc $C --output-format csv -d "$O/${TAG}_pmc_$C" -o pmc -- $B --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5
      done
      (cd /tmp && run pmc_MFMA 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/${TAG}_pmc_MFMA" -o pmc -- $B --lanes 1 --steps 1 --warmup 0 --decode-steps 8 --no-cpu-baseline) || exit 5 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all steps done"
