#!/bin/bash
# One GPU-box pass: parity suite, bench line, rocprofv3 kernel stats of the bench, and HBM-traffic
# PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs) on the quantize forward.
#   gpurun --timeout 1100 -- bash tools/gpu_check.sh [tests|bench|prof|pmc ...]
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
steps="${*:-tests bench prof pmc}"
export TMPDIR=/tmp

run() {   # name, seconds, command...
  local name="$1" secs="$2"; shift 2
  echo "[$(date +%T)] $name: $*" >&2
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "[$(date +%T)] $name exit $rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}

for s in $steps; do
  case "$s" in
    tests)
      run tests 600 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1 || exit 1
      tail -3 "$O/gpu_tests.log" ;;
    gemmtests)   # split-K / accumulate / direct-grad GEMM parity only
      run gemmtests 300 python -u -m pytest "$R/tests/test_gemm_splitk_epi_gpu.py" "$R/tests/test_gemm_x3s_gpu.py" \
        "$R/tests/test_direct_grad_gpu.py" "$R/tests/test_gemm_bf16x3_gpu.py" -m gpu -x -q --timeout 120 \
        --timeout-method thread > "$O/gemmtests.log" 2>&1 || { tail -30 "$O/gemmtests.log"; exit 1; }
      tail -3 "$O/gemmtests.log" ;;
    hoisttests)   # hoisted K/V projection + decoder paths it touches
      run hoisttests 400 python -u -m pytest "$R/tests/test_direct_grad_gpu.py" "$R/tests/test_train_gpu.py" \
        "$R/tests/test_reference_fixtures_gpu.py" "$R/tests/test_fused_decoder_gpu.py" "$R/tests/test_jagged_attention_gpu.py" -m gpu -x -q --timeout 120 \
        --timeout-method thread > "$O/hoisttests.log" 2>&1 || { tail -40 "$O/hoisttests.log"; exit 1; }
      tail -3 "$O/hoisttests.log" ;;
    abhoist)
      run abhoist 400 python -u "$R/tools/ab_hoist.py" hoist 2 > "$O/abhoist.jsonl" 2> "$O/abhoist.err"
      tail -1 "$O/abhoist.jsonl" ;;
    rqside)
      run rqside 200 python -u "$R/tools/rq_side_ab.py" 20 3 > "$O/rqside.jsonl" 2> "$O/rqside.err"
      cat "$O/rqside.jsonl" ;;
    bench)
      run bench 400 python -u "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
      cat "$O/bench.json" ;;
    prof)
      cd /tmp
      run prof 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o bench -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-pmc > "$O/prof_bench.json" 2> "$O/prof_bench.err"
      run prof_rq 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o rqvae -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-pmc --no-extras > "$O/prof_rqvae.json" 2> "$O/prof_rqvae.err"
      run prof_dec 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o decoder -- \
        python3 "$R/bench.py" --decoder-only > "$O/prof_decoder.json" 2> "$O/prof_decoder.err"
      cd "$R"
      cat "$O/prof_bench.json" ;;
    pmc)
      cd /tmp
      run pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rq_fwd -f csv -d "$O/pmc_fetch" -o q -- \
        python3 "$R/tools/pmc_quantize.py" 10 > "$O/pmc_fetch.log" 2>&1
      run pmc_write 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rq_fwd -f csv -d "$O/pmc_write" -o q -- \
        python3 "$R/tools/pmc_quantize.py" 10 > "$O/pmc_write.log" 2>&1
      cd "$R" ;;
    profdec)
      cd /tmp
      run prof_dec 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o decoder -- \
        python3 "$R/bench.py" --decoder-only > "$O/prof_decoder.json" 2> "$O/prof_decoder.err"
      cd "$R"
      cat "$O/prof_decoder.json" ;;
    profdm8)   # C4 per-rank config: ML-32M decoder, 8 sequences per GPU
      cd /tmp
      run prof_dm8 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o dm8 -- \
        python3 "$R/bench.py" --decoder-only --dm-batch 8 > "$O/prof_dm8.json" 2> "$O/prof_dm8.err"
      cd "$R"
      cat "$O/prof_dm8.json" ;;
    attnab)   # short-form attention: LDS-DMA kernels on (default) vs off, Amazon / cross shapes
      run attn_dma1 200 python -u "$R/tools/attn_probe.py" > "$O/attn_dma1.jsonl" 2> "$O/attn_dma1.err"
      RQ_ATTN_DMA=0 run attn_dma0 200 python -u "$R/tools/attn_probe.py" > "$O/attn_dma0.jsonl" 2> "$O/attn_dma0.err"
      grep -h amazon "$O/attn_dma1.jsonl" "$O/attn_dma0.jsonl" ;;
    libprobe)   # library bf16 GEMM over a tripled k vs the split-bf16 kernels at decoder shapes
      run libprobe 200 python -u "$R/tools/lib_bf16_probe.py" 20 > "$O/libprobe.jsonl" 2> "$O/libprobe.err"
      cat "$O/libprobe.jsonl" ;;
    sqdec)   # SQ counter passes on the decoder's qkv forward (fp32 A) and qkv dgrad shapes
      run sq_qkv 150 bash "$R/tools/pmc_sq_gemm.sh" 11264 1536 512 1 1 0 1 qkv_fwd
      run sq_dgrad 150 bash "$R/tools/pmc_sq_gemm.sh" 11264 512 1536 1 0 0 1 qkv_dgrad
      run sq_fc1w 150 bash "$R/tools/pmc_sq_gemm.sh" 11264 1024 512 1 1 1 1 fc1_wide ;;
    attntests)   # attention kernels + the decoder fixtures
      run attntests 400 python -u -m pytest "$R/tests/test_jagged_attention_gpu.py" "$R/tests/test_reference_fixtures_gpu.py" \
        -m gpu -x -q --timeout 120 --timeout-method thread > "$O/attntests.log" 2>&1 || { tail -40 "$O/attntests.log"; exit 1; }
      tail -3 "$O/attntests.log" ;;
    fewqab)   # one-pass few-query backward on / off: attention probe + decoder Amazon step
      RQ_ATTN_FEWQ_FUSED=1 run fewq1 200 python -u "$R/tools/attn_probe.py" > "$O/fewq1.jsonl" 2> "$O/fewq1.err"
      RQ_ATTN_FEWQ_FUSED=0 run fewq0 200 python -u "$R/tools/attn_probe.py" > "$O/fewq0.jsonl" 2> "$O/fewq0.err"
      grep -h cross "$O/fewq1.jsonl" "$O/fewq0.jsonl"
      RQ_ATTN_FEWQ_FUSED=1 run dec1 200 python -u "$R/bench.py" --decoder-only > "$O/dec_fewq1.json" 2> "$O/dec_fewq1.err"
      RQ_ATTN_FEWQ_FUSED=0 run dec0 200 python -u "$R/bench.py" --decoder-only > "$O/dec_fewq0.json" 2> "$O/dec_fewq0.err"
      RQ_ATTN_FEWQ_FUSED=1 run dec1b 200 python -u "$R/bench.py" --decoder-only > "$O/dec_fewq1b.json" 2> "$O/dec_fewq1b.err"
      cat "$O/dec_fewq1.json" "$O/dec_fewq0.json" "$O/dec_fewq1b.json" | python3 -c "import sys,json; [print(json.loads(l)['decoder_amazon']['ms_per_step']) for l in sys.stdin]" ;;
    shortab)   # one-pass short self-attention backward on / off: decoder Amazon step (alternating)
      for v in 1 0 1 0; do
        RQ_ATTN_SHORT_FUSED=$v run dec_s$v 200 python -u "$R/bench.py" --decoder-only > "$O/dec_short$v.json" 2> "$O/dec_short$v.err"
        python3 -c "import json; print('short_fused=$v', json.load(open('$O/dec_short$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    x3dtests)
      run x3dtests 300 python -u -m pytest "$R/tests/test_gemm_x3d_gpu.py" "$R/tests/test_gemm_bf16x3_gpu.py" "$R/tests/test_gemm_splitk_epi_gpu.py" \
        -m gpu -x -q --timeout 120 --timeout-method thread > "$O/x3dtests.log" 2>&1 || { tail -40 "$O/x3dtests.log"; exit 1; }
      tail -3 "$O/x3dtests.log" ;;
    x3dab)   # LDS-DMA 128-tile form on / off: decoder Amazon step (alternating) + library probe shapes
      for v in 1 0 1 0; do
        RQ_X3D=$v run dec_d$v 200 python -u "$R/bench.py" --decoder-only > "$O/dec_x3d$v.json" 2> "$O/dec_x3d$v.err"
        python3 -c "import json; print('x3d=$v', json.load(open('$O/dec_x3d$v.json'))['decoder_amazon']['ms_per_step'])"
      done
      RQ_X3D=1 run libx3d1 200 python -u "$R/tools/lib_bf16_probe.py" 20 > "$O/lib_x3d1.jsonl" 2> "$O/lib_x3d1.err"
      RQ_X3D=0 run libx3d0 200 python -u "$R/tools/lib_bf16_probe.py" 20 > "$O/lib_x3d0.jsonl" 2> "$O/lib_x3d0.err"
      python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
a = [json.loads(l) for l in open(o + "/lib_x3d1.jsonl")]
b = [json.loads(l) for l in open(o + "/lib_x3d0.jsonl")]
for x, y in zip(a, b):
    print(x["shape"], "fp32A x3d", x["x3_fp32A_splitB_us"], "staged", y["x3_fp32A_splitB_us"], "split", x["x3_split_us"])
PY
      ;;
    redab)   # split-K reduction-launch cost in the GEMM planner: decoder Amazon + ML-32M B=8 steps
      for v in 4 7 10 4 7 10; do
        RQ_X3_REDUCE_US=$v run dec_r$v 200 python -u "$R/bench.py" --decoder-only > "$O/dec_red$v.json" 2> "$O/dec_red$v.err"
        RQ_X3_REDUCE_US=$v run dm8_r$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_red$v.json" 2> "$O/dm8_red$v.err"
        python3 -c "import json; print('reduce_us=$v amazon', json.load(open('$O/dec_red$v.json'))['decoder_amazon']['ms_per_step'], 'dm8', json.load(open('$O/dm8_red$v.json'))['decoder_ml32m']['ms_per_step'])"
      done ;;
    qsplitab)   # fused attention backward query split at the C4 per-rank config (ML-32M, 8 sequences)
      for v in 0 6 8 4 0 6 8; do
        RQ_ATTN_QSPLIT=$v run dm8_q$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_q$v.json" 2> "$O/dm8_q$v.err"
        python3 -c "import json; print('qsplit=$v dm8', json.load(open('$O/dm8_q$v.json'))['decoder_ml32m']['ms_per_step'])"
      done ;;
    hoistab)   # hoisted cross K/V projection with its input split once (RQ_HOIST_SPLIT) on / off
      for v in 1 0 1 0; do
        RQ_HOIST_SPLIT=$v run dec_h$v 200 python -u "$R/bench.py" --decoder-only > "$O/dec_hs$v.json" 2> "$O/dec_hs$v.err"
        python3 -c "import json; print('hoist_split=$v', json.load(open('$O/dec_hs$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    kvsplitab)   # key-split forward (RQ_ATTN_KVSPLIT) on / off at the C4 per-rank config
      for v in 1 0 1 0; do
        RQ_ATTN_KVSPLIT=$v run dm8_k$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_k$v.json" 2> "$O/dm8_k$v.err"
        python3 -c "import json; print('kvsplit=$v dm8', json.load(open('$O/dm8_k$v.json'))['decoder_ml32m']['ms_per_step'])"
      done ;;
    wsab)   # weight gradients on a side stream (--wgrad-stream) at both decoder configs
      for v in 1 0 1 0; do
        f=""; [ $v = 1 ] && f="--wgrad-stream"
        run dm8_ws$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 $f > "$O/dm8_ws$v.json" 2> "$O/dm8_ws$v.err"
        run am_ws$v 200 python -u "$R/bench.py" --decoder-only $f > "$O/am_ws$v.json" 2> "$O/am_ws$v.err"
        python3 -c "import json; print('wgrad_stream=$v dm8', json.load(open('$O/dm8_ws$v.json'))['decoder_ml32m']['ms_per_step'], 'amazon', json.load(open('$O/am_ws$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    ceab)   # fused loss head (RQ_FUSED_CE) tests + on / off at both decoder configs
      run cetests 200 python -u -m pytest "$R/tests/test_ce_loss_gpu.py" "$R/tests/test_reference_fixtures_gpu.py" "$R/tests/test_train_gpu.py" \
        -m gpu -x -q --timeout 120 --timeout-method thread > "$O/cetests.log" 2>&1 || { tail -40 "$O/cetests.log"; exit 1; }
      tail -1 "$O/cetests.log"
      for v in 1 0 1 0; do
        RQ_FUSED_CE=$v run dm8_c$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_c$v.json" 2> "$O/dm8_c$v.err"
        RQ_FUSED_CE=$v run am_c$v 200 python -u "$R/bench.py" --decoder-only > "$O/am_c$v.json" 2> "$O/am_c$v.err"
        python3 -c "import json; print('fused_ce=$v dm8', json.load(open('$O/dm8_c$v.json'))['decoder_ml32m']['ms_per_step'], 'amazon', json.load(open('$O/am_c$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    pairprobe)   # dgrad + wgrad back to back vs concurrent (two streams)
      run pairprobe 200 python -u "$R/tools/pair_probe.py" 50 > "$O/pairprobe.jsonl" 2> "$O/pairprobe.err"
      cat "$O/pairprobe.jsonl" ;;
    trainers)   # drop-in trainers: GPU tests + their own steady-state timing
      run trtests 400 python -u -m pytest "$R/tests/test_train_gpu.py" -m gpu -x -q --timeout 200 --timeout-method thread \
        > "$O/trtests.log" 2>&1 || { tail -40 "$O/trtests.log"; exit 1; }
      tail -1 "$O/trtests.log"
      run trprobe 300 python -u "$R/tools/trainer_probe.py" > "$O/trainers.json" 2> "$O/trainers.err"
      cat "$O/trainers.json" ;;
    pairab)   # paired dgrad/wgrad launches: tests, then on / off at both decoder configs
      run pairtests 400 python -u -m pytest "$R/tests/test_gemm_pair_gpu.py" "$R/tests/test_direct_grad_gpu.py" "$R/tests/test_fused_decoder_gpu.py" \
        "$R/tests/test_reference_fixtures_gpu.py" "$R/tests/test_mlp_recon_gpu.py" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pairtests.log" 2>&1 \
        || { tail -40 "$O/pairtests.log"; exit 1; }
      tail -1 "$O/pairtests.log"
      for v in 1 0 1 0; do
        RQ_X3_PAIR=$v run dm8_p$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_p$v.json" 2> "$O/dm8_p$v.err"
        RQ_X3_PAIR=$v run am_p$v 200 python -u "$R/bench.py" --decoder-only > "$O/am_p$v.json" 2> "$O/am_p$v.err"
        python3 -c "import json; print('pair=$v dm8', json.load(open('$O/dm8_p$v.json'))['decoder_ml32m']['ms_per_step'], 'amazon', json.load(open('$O/am_p$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    tpwab)   # short fused attention backward: one key tile per wave (default) vs 4 waves x 2 tiles
      for v in 1 2 1 2; do
        RQ_ATTN_SHORT_TPW=$v run am_t$v 200 python -u "$R/bench.py" --decoder-only > "$O/am_t$v.json" 2> "$O/am_t$v.err"
        python3 -c "import json; print('short_tpw=$v amazon', json.load(open('$O/am_t$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    kfullab)   # unmasked GEMM staging (RQ_X3_KFULL) on / off: tests, then the decoder configs and the RQ-VAE line
      run kftests 500 python -u -m pytest "$R/tests/test_gemm_kfull_gpu.py" "$R/tests/test_gemm_pair_gpu.py" "$R/tests/test_gemm_bf16x3_gpu.py" \
        "$R/tests/test_gemm_x3s_gpu.py" "$R/tests/test_reference_fixtures_gpu.py" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/kftests.log" 2>&1 \
        || { tail -40 "$O/kftests.log"; exit 1; }
      tail -1 "$O/kftests.log"
      for v in 1 0 1 0; do
        RQ_X3_KFULL=$v run dm8_k$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_k$v.json" 2> "$O/dm8_k$v.err"
        RQ_X3_KFULL=$v run am_k$v 200 python -u "$R/bench.py" --decoder-only > "$O/am_k$v.json" 2> "$O/am_k$v.err"
        RQ_X3_KFULL=$v run rq_k$v 200 python -u "$R/bench.py" --no-cpu-baseline --no-pmc --no-extras > "$O/rq_k$v.json" 2> "$O/rq_k$v.err"
        python3 -c "import json; print('kfull=$v dm8', json.load(open('$O/dm8_k$v.json'))['decoder_ml32m']['ms_per_step'], 'amazon', json.load(open('$O/am_k$v.json'))['decoder_amazon']['ms_per_step'], 'rqvae', json.load(open('$O/rq_k$v.json'))['ms_per_step'])"
      done ;;
    embab)   # batched (deferred) embedding-table gradients on / off
      run embtests 400 python -u -m pytest "$R/tests/test_direct_grad_gpu.py" "$R/tests/test_fused_decoder_gpu.py" "$R/tests/test_reference_fixtures_gpu.py" \
        "$R/tests/test_graph_gpu.py" "$R/tests/test_train_gpu.py" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/embtests.log" 2>&1 \
        || { tail -40 "$O/embtests.log"; exit 1; }
      tail -1 "$O/embtests.log"
      for v in 1 0 1 0; do
        RQ_EMB_DEFER=$v run dm8_e$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_e$v.json" 2> "$O/dm8_e$v.err"
        RQ_EMB_DEFER=$v run am_e$v 200 python -u "$R/bench.py" --decoder-only > "$O/am_e$v.json" 2> "$O/am_e$v.err"
        python3 -c "import json; print('emb_defer=$v dm8', json.load(open('$O/dm8_e$v.json'))['decoder_ml32m']['ms_per_step'], 'amazon', json.load(open('$O/am_e$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    unsplitab)   # paired data gradient unsplit (RQ_X3_PAIR_UNSPLIT) on / off
      run pairtests2 300 python -u -m pytest "$R/tests/test_gemm_pair_gpu.py" "$R/tests/test_reference_fixtures_gpu.py" "$R/tests/test_direct_grad_gpu.py" \
        -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pairtests2.log" 2>&1 || { tail -40 "$O/pairtests2.log"; exit 1; }
      tail -1 "$O/pairtests2.log"
      for v in 1 0 1 0; do
        RQ_X3_PAIR_UNSPLIT=$v run dm8_u$v 200 python -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_u$v.json" 2> "$O/dm8_u$v.err"
        RQ_X3_PAIR_UNSPLIT=$v run am_u$v 200 python -u "$R/bench.py" --decoder-only > "$O/am_u$v.json" 2> "$O/am_u$v.err"
        python3 -c "import json; print('pair_unsplit=$v dm8', json.load(open('$O/dm8_u$v.json'))['decoder_ml32m']['ms_per_step'], 'amazon', json.load(open('$O/am_u$v.json'))['decoder_amazon']['ms_per_step'])"
      done ;;
    keysdm8)   # per-shape device times (and GEMM plans) of one ML-32M decoder step at 8 sequences
      run keys_dm8 200 python -u "$R/tools/dec_gemm_keys.py" 5 dm8 > "$O/keys_dm8.jsonl" 2> "$O/keys_dm8.err"
      tail -1 "$O/keys_dm8.jsonl" ;;
    keys)    # per-shape device times of the RQ-VAE step and of one decoder step (HIP events)
      run keys_rq 200 python -u "$R/tools/gemm_keys.py" 5 > "$O/keys_rq.jsonl" 2> "$O/keys_rq.err"
      run keys_dec 200 python -u "$R/tools/dec_gemm_keys.py" 5 > "$O/keys_dec.jsonl" 2> "$O/keys_dec.err"
      tail -1 "$O/keys_rq.jsonl"; tail -1 "$O/keys_dec.jsonl" ;;
    attnab2)   # same-process, alternating A/B of the attention forms at the Amazon decoder shapes
      run attnab2 200 python -u "$R/tools/attn_ab2.py" 20 3 > "$O/attnab2.jsonl" 2> "$O/attnab2.err"
      cat "$O/attnab2.jsonl" ;;
    epiab)   # wide GEMM kernel with / without its epilogue (diagnostic build build_ab/x3w_noepi.so)
      GEMM_AB_KERNELS=wide GEMM_AB_CASES="enc0,dec3 fwd,dec-ctx" run epiab_a 200 python -u "$R/tools/gemm_ab.py" 20 > "$O/epiab_a.jsonl" 2>&1
      RQVAE_HIP_LIB="$R/build_ab/x3w_noepi.so" GEMM_AB_KERNELS=wide GEMM_AB_CASES="enc0,dec3 fwd,dec-ctx" run epiab_b 200 python -u "$R/tools/gemm_ab.py" 20 > "$O/epiab_b.jsonl" 2>&1
      grep -h '"us"' "$O/epiab_a.jsonl" "$O/epiab_b.jsonl" ;;
    decgemm)   # decoder context-row GEMM operand forms / kernels (tools/dec_gemm_probe.py)
      run decgemm 200 python -u "$R/tools/dec_gemm_probe.py" 20 > "$O/decgemm.jsonl" 2> "$O/decgemm.err"
      cat "$O/decgemm.jsonl" ;;
    sqpmc)
      cd /tmp
      run pmc_sq 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
        --kernel-include-regex "rq_fwd|rq_dist" -f csv -d "$O/pmc_sq" -o q -- python3 "$R/tools/pmc_quantize.py" 5 > "$O/pmc_sq.log" 2>&1
      run pmc_sq2 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE \
        --kernel-include-regex "rq_fwd|rq_dist" -f csv -d "$O/pmc_sq2" -o q -- python3 "$R/tools/pmc_quantize.py" 5 > "$O/pmc_sq2.log" 2>&1
      cd "$R" ;;
    attnprof)   # kernel-level A/B of the attention forms (attn_ab2 alternates DMA / few-query forms on and off)
      cd /tmp
      run attnprof 200 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o attnab -- \
        python3 "$R/tools/attn_ab2.py" 20 2 > "$O/attnprof.log" 2>&1
      cd "$R" ;;
    attnpmc)   # SQ counters of the Amazon-shape attention kernels (tools/attn_ab2.py, DMA forms on)
      cd /tmp
      run pmc_attn1 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
        --kernel-include-regex "attn_" -f csv -d "$O/pmc_attn1" -o a -- python3 "$R/tools/attn_ab2.py" 2 1 > "$O/pmc_attn1.log" 2>&1
      run pmc_attn2 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE \
        --kernel-include-regex "attn_" -f csv -d "$O/pmc_attn2" -o a -- python3 "$R/tools/attn_ab2.py" 2 1 > "$O/pmc_attn2.log" 2>&1
      cd "$R" ;;
    dp2)   # two ranks sharing the one GPU over gloo: exercises every multi-rank code path of bench.py
      RQVAE_DIST_BACKEND=gloo RQVAE_SHARE_DEVICE=1 run dp2 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 "$R/bench.py" --gpus 2 --steps 5 --warmup 3 \
        > "$O/bench_dp2.json" 2> "$O/bench_dp2.err"
      cat "$O/bench_dp2.json" ;;
    kern)
      run kern 300 python -u "$R/tools/bench_kernels.py" > "$O/kernels.jsonl" 2> "$O/kernels.err"
      cat "$O/kernels.jsonl" ;;
    gemm3)
      run gemm3_tests 300 python -u -m pytest "$R/tests/test_gemm_bf16x3_gpu.py" -m gpu -x -q --timeout 120 \
        --timeout-method thread > "$O/gemm3_tests.log" 2>&1 || { tail -30 "$O/gemm3_tests.log"; exit 1; }
      tail -3 "$O/gemm3_tests.log"
      run gemm3 200 python -u "$R/tools/bench_kernels.py" --gemm3 > "$O/gemm3.jsonl" 2> "$O/gemm3.err"
      cat "$O/gemm3.jsonl" ;;
    wgrad)
      run wgrad 200 python -u "$R/tools/bench_kernels.py" --wgrad > "$O/wgrad.jsonl" 2> "$O/wgrad.err"
      cat "$O/wgrad.jsonl"
      cd /tmp
      run prof_wgrad 200 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o wgrad -- \
        python3 "$R/tools/bench_kernels.py" --wgrad --rounds 3 > "$O/prof_wgrad.log" 2>&1
      cd "$R" ;;
    abopt)   # same box, alternating: HIP multi-tensor AdamW (A) vs torch fused AdamW (B)
      for k in 1 2; do
        run abopt_A$k 200 python -u "$R/bench.py" --no-cpu-baseline --no-pmc > "$O/abopt_A$k.json" 2> "$O/abopt.err"
        RQVAE_TORCH_ADAMW=1 run abopt_B$k 200 python -u "$R/bench.py" --no-cpu-baseline --no-pmc > "$O/abopt_B$k.json" 2>> "$O/abopt.err"
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
