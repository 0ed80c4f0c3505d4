#!/bin/bash
# Round-5 GPU recipes (one function per measurement; outputs under gpurun_out/, the kept ones
# copied to profiles/r05/). Run from the repo root, on the GPU box:
#   bash tools/r05_runs.sh <recipe> [args]
# Recipes:
#   attn       Round 5: the persistent attention pair loop (attention_pp_kernel) — kernel tests, attention timing, then a same-box A/B against the previous build (ab/base.so). Output gpurun_out/r05_attn/.
#   blas_prof  r05: which hipBLASLt kernels (macro tile, depth) run the B/32 shapes
#   check      Round 5: GEMM kernel tests of variant 72 / blocked W after the header clean-up, then the reference-harness fixtures. Output under gpurun_out/r05_check/.
#   final_ab   Round 5 closing A/B of the shipped defaults against the r04 GEMM defaults, per config.
#   fold       Round 5: the LayerNorm fold on the 24-bit residual stream — parity tests, then the same-box A/B against the shipped default and the fp32-x fold. Output under gpurun_out/r05_fold/.
#   fold_prof  Round 5: per-role kernel trace + FETCH_SIZE / WRITE_SIZE passes of the shipped default and of the LayerNorm fold on the 24-bit stream (tuning lnfold=1), same box. Summaries are made on the host: python tools/summarize_profiles.py gpurun_out/r05_foldprof/<arm> r05_fold_<arm> 256 --summary-only
#   golden     Round 5: the reference-harness fixtures (flat + CLIP-scale) with the literal rank-1 rule; prints the per-case worst relative logit error. Output under gpurun_out/r05_golden/.
#   kt         Kernel-trace stats of the default bench against tuning arms (per-kernel average durations). bash tools/r05_runs.sh kt OUTDIR "<tuning spec>" ...   ("-" = the shipped default)
#   large      Round 5: the large-M roles on variant 72 + blocked W (new default) — race screen, bit-identity and parity tests, then same-box A/B against the r04 large-M defaults on L/14@336, B/16 and B/32. Output under gpurun_out/r05_large/.
#   layout     Round 5: variant 72 operand layout / k-rotation experiments on c_fc main and QKV (tools/probes/gemm_probe p32). Output under gpurun_out/r05_p32/.
#   mx_epi     r05: MX-fp8 tile costs by epilogue (store16 vs QuickGELU + quantize) against the 16-bit tiles
#   nt         Round 5: variant 74 (72 with non-temporal stores) for the large-M c_fc — tests, then A/B on B/16 and L/14@336 against the shipped 3472 c_fc. Output under gpurun_out/r05_nt/.
#   p32        Round 5: variant 72 (gemm_p32.h) — kernel correctness tests, then interleaved kernel A/B against the shipped tiles on the B/32 bs-256 shapes and 4096^3. Output under gpurun_out/r05_p32/.
#   pmc        Round 5: PMC passes (one counter set per rocprofv3 run, --kernel-trace + --pmc only) of the QKV shape on v72 (row-major / blocked operands) and the v62 copy, and of c_proj's shipped tile (v82 via tools/gemm_ab.py). Output under gpurun_out/r05_pmc/<kind>/.
#   pmc2       Round 5: LDS / instruction-issue PMC passes of variant 72 (QKV shape, row-major and blocked operands) and the v62 copy. Output under gpurun_out/r05_pmc2/.
#   probe      Round-5 GEMM timeline probe (tools/probes/gemm_probe.hip): barrier / MFMA-segment micro-probe, then the stamped persistent ping-pong on the B/32 bs-256 shapes. Output under gpurun_out/.
#   seg        Round-5 ping-pong segment-cost micro-probe (tools/probes/gemm_probe bar). Output under gpurun_out/.
#   v62blk     r05: blocked weight copy on the persistent ping-pong tile (v62/63): kernel screens + same-box A/B against the previous default (blocked W on the pipelined and 32-deep tiles only).
#   w73        Round 5: blocked weight operand (GemmArgs.blk_w, tuning w_blocked) on the pipelined tiles and variant 72 — kernel tests, bit-identity in the model, in-model A/B. Output under gpurun_out/r05_w73/.
#   yardstick  r05: hipBLASLt (torch linear) against the library's tiles on the B/32 shapes, same box
set -o pipefail

run_attn() {
  out=gpurun_out/r05_attn
  mkdir -p $out
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "attention_pair" > $out/tests.log 2>&1 || { echo "attention tests failed"; tail -30 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
  timeout -k 10 120 python -u tools/attn_probe.py 256,50,12 > $out/probe_new.log 2>&1 || { echo probe failed; tail -5 $out/probe_new.log; exit 1; }
  CLIPVIT_LIB=$PWD/abase/base.so timeout -k 10 120 python -u tools/attn_probe.py 256,50,12 > $out/probe_base.log 2>&1 || { echo probe failed; exit 1; }
  echo "new: $(cat $out/probe_new.log | tail -1)"; echo "base: $(cat $out/probe_base.log | tail -1)"
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "CLIPVIT_LIB=$PWD/abase/base.so" > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
}

run_blas_prof() {
  out=$PWD/gpurun_out/r05_blas_prof
  mkdir -p $out
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/blas_yardstick.py --dtypes float16 --iters 20 > $out/log.txt 2>&1 || { echo "prof failed"; tail -5 $out/log.txt; exit 1; }
  find $out/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-400
}

run_check() {
  out=gpurun_out/r05_check
  mkdir -p $out
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "gemm and (72 or 100)" > $out/kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 $out/kernels.log; exit 1; }
  tail -1 $out/kernels.log
  run_golden
}

run_final_ab() {
  out=gpurun_out/r05_final_ab
  mkdir -p $out
  OLD="--tuning w_blocked=0;split_variants=62,81;large_variants=3462,3463,3463,3463"
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "$OLD" > $out/b32.log 2>&1 || { echo "b32 A/B failed"; tail -5 $out/b32.log; exit 1; }
  bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "$OLD" > $out/b16.log 2>&1 || { echo "b16 A/B failed"; exit 1; }
  bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" 2 - "$OLD" > $out/l14.log 2>&1 || { echo "l14 A/B failed"; exit 1; }
  cat $out/b32.log $out/b16.log $out/l14.log | cut -c1-120
}

run_fold() {
  out=gpurun_out/r05_fold
  mkdir -p $out
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "lnfold or cls_prune_and_deferred or blocked_u_is_bit_identical" -s > $out/parity.log 2>&1 \
    || { echo "parity failed"; tail -40 $out/parity.log; exit 1; }
  grep -E "passed|failed|rel |err " $out/parity.log | tail -30
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning lnfold=1" "--tuning lnfold=1;x24=0" \
    > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
}

run_fold_prof() {
  set -e
  ROOT=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  for arm in def fold; do
    OUT=$ROOT/gpurun_out/r05_foldprof/$arm
    mkdir -p $OUT
    X=(); [ $arm = fold ] && X=(--tuning lnfold=1)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run \
      -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --profile-iters 2 "${X[@]}" > $OUT/kt.log 2>&1
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run \
      -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --profile-iters 1 "${X[@]}" > $OUT/fetch.log 2>&1
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run \
      -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --profile-iters 1 "${X[@]}" > $OUT/write.log 2>&1
    echo "$arm done"
  done
}

run_golden() {
  out=gpurun_out/r05_golden
  mkdir -p $out
  timeout -k 10 500 python -u -m pytest tests/test_gpu_golden.py -x -v --timeout 400 --timeout-method thread \
    -k "flat_fixtures or clipscale_harness" -s > $out/golden.log 2>&1 \
    || { echo "golden failed"; grep -E "rel logit|swaps|Error|assert" $out/golden.log | tail -30; exit 1; }
  grep -E "rel logit|swaps|argmax|passed|failed" $out/golden.log
}

run_kt() {
  set -e
  OUT=$1; shift
  ROOT=$(pwd)
  mkdir -p "$OUT"
  cd /tmp && export TMPDIR=/tmp
  i=0
  for arm in "$@"; do
    X=()
    [ "$arm" != "-" ] && X=(--tuning "$arm")
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt$i" -o run \
      -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline "${X[@]}" > "$ROOT/$OUT/kt$i.log" 2>&1
    echo "arm $i: $arm" >> "$ROOT/$OUT/arms.txt"
    i=$((i+1))
  done
  echo kt-done
}

run_large() {
  out=gpurun_out/r05_large
  mkdir -p $out
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread -k "p32_race or blocked_w or blocked_u or L14 or l14 or large" > $out/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
  OLD="--tuning w_blocked=0;large_variants=3462,3463,3463,3463"
  bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" 2 - "$OLD" > $out/l14.log 2>&1 \
    || { echo "l14 A/B failed"; tail -5 $out/l14.log; exit 1; }
  bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "$OLD" > $out/b16.log 2>&1 \
    || { echo "b16 A/B failed"; tail -5 $out/b16.log; exit 1; }
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "$OLD" > $out/b32.log 2>&1 || { echo "b32 A/B failed"; tail -5 $out/b32.log; exit 1; }
  cat $out/l14.log $out/b16.log $out/b32.log | cut -c1-150
}

run_layout() {
  out=gpurun_out/r05_p32
  mkdir -p $out
  { echo "== c_fc main 10752x3072x768 gelu xcd34"; timeout -k 10 60 tools/probes/gemm_probe p32 10752 3072 768 1 34 && \
    echo "== QKV 12800x2304x768 xcd0"; timeout -k 10 60 tools/probes/gemm_probe p32 12800 2304 768 0 0; } > $out/layout3.log 2>&1 \
    || { echo "layout probe failed"; tail -20 $out/layout3.log; exit 1; }
  grep -v "^  step\|^tile\|epilogue of" $out/layout3.log
}

run_mx_epi() {
  out=gpurun_out/r05_mx_epi
  mkdir -p $out
  GEMM_AB_DTYPE=3 timeout -k 10 300 python -u tools/gemm_ab.py "12800,3072,768,0;12800,3072,768,1;12800,2304,768,0;12800,768,3072,0" "3,1,2" 5 20 > $out/mx.log 2>&1 || { echo "mx failed"; tail -5 $out/mx.log; exit 1; }
  GEMM_AB_DTYPE=2 timeout -k 10 300 python -u tools/gemm_ab.py "12800,3072,768,0;12800,3072,768,1;12800,2304,768,0;12800,768,3072,0" "62,72,10072" 5 20 > $out/f16.log 2>&1 || { echo "f16 failed"; tail -5 $out/f16.log; exit 1; }
  cat $out/mx.log $out/f16.log
}

run_nt() {
  out=gpurun_out/r05_nt
  mkdir -p $out
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
    -k "(gemm and 74) or p32_race" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
  bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "--tuning large_variants=3462,3474,3463,3463" > $out/b16.log 2>&1 \
    || { echo "b16 A/B failed"; tail -5 $out/b16.log; exit 1; }
  bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" 2 - "--tuning large_variants=3472,3474,3472,3472" > $out/l14.log 2>&1 \
    || { echo "l14 A/B failed"; tail -5 $out/l14.log; exit 1; }
  cat $out/b16.log $out/l14.log | cut -c1-230
}

run_p32() {
  out=gpurun_out/r05_p32
  mkdir -p $out
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "72" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
  timeout -k 10 300 python -u tools/gemm_ab.py "10752,3072,768,1;12800,3072,768,1;12800,2304,768,0;4096,4096,4096,0" \
    "3462,3472,62,72" 5 20 > $out/ab.log 2>&1 || { echo "ab failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
  # in-model: the shipped line against v72 as the c_fc main launch, and also as the QKV tile
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning split_variants=72,81" \
    "--tuning split_variants=72,81;qkv_variant=72" > $out/inmodel.log 2>&1 || { echo "in-model A/B failed"; tail -20 $out/inmodel.log; exit 1; }
  cat $out/inmodel.log
}

run_pmc() {
  cd /tmp && export TMPDIR=/tmp
  R=$GRAFT_REPO_ROOT
  out=$R/gpurun_out/r05_pmc
  mkdir -p $out
  for kind in 0 1 2 cproj; do
    if [ $kind = cproj ]; then P="python3 $R/tools/gemm_ab.py 12800,768,3072,0 82 1 30"
    else P="$R/tools/probes/gemm_probe p32run 12800 2304 768 0 0 30 $kind"; fi
    i=0
    for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
               "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $out/k$kind/p$i -o run -- $P > $out/k$kind.p$i.log 2>&1 \
        || { rc=$?; echo "kind $kind pass $i ($set) failed rc=$rc"; tail -3 $out/k$kind.p$i.log; [ $rc -ge 124 ] && exit 1; }
    done
  done
  echo done
}

run_pmc2() {
  cd /tmp && export TMPDIR=/tmp
  R=$GRAFT_REPO_ROOT
  out=$R/gpurun_out/r05_pmc2
  mkdir -p $out
  for kind in 0 1 2; do
    P="$R/tools/probes/gemm_probe p32run 12800 2304 768 0 0 30 $kind"
    i=0
    for set in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
               "SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM" \
               "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $out/k$kind/p$i -o run -- $P > $out/k$kind.p$i.log 2>&1 \
        || { rc=$?; echo "kind $kind pass $i ($set) failed rc=$rc"; tail -3 $out/k$kind.p$i.log; [ $rc -ge 124 ] && exit 1; }
    done
  done
  echo done
}

run_probe() {
  out=gpurun_out/r05_probe
  mkdir -p $out
  P=tools/probes/gemm_probe
  run() { echo "== $*"; timeout -k 10 120 $P "$@"; }
  {
  run bar && \
  run 10752 3072 768 1 34 && \
  run 12800 2304 768 0 0
  } > $out/probe2.txt 2>&1 || { echo "probe failed"; tail -30 $out/probe2.txt; exit 1; }
  head -12 $out/probe2.txt
}

run_seg() {
  mkdir -p gpurun_out/r05_probe
  timeout -k 10 120 tools/probes/gemm_probe bar > gpurun_out/r05_probe/seg.txt 2>&1 || { tail -20 gpurun_out/r05_probe/seg.txt; exit 1; }
  cat gpurun_out/r05_probe/seg.txt
}

run_v62blk() {
  out=gpurun_out/r05_v62blk
  mkdir -p $out
  timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -m gpu -k "race_screen or blocked or gemm_shapes" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
  tail -3 $out/tests.log
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning w_blocked=1" > $out/b32.log 2>&1 || { echo "b32 A/B failed"; tail -5 $out/b32.log; exit 1; }
  bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "--tuning w_blocked=1" > $out/b16.log 2>&1 || { echo "b16 A/B failed"; exit 1; }
  cat $out/b32.log $out/b16.log | cut -c1-140
}

run_w73() {
  out=gpurun_out/r05_w73
  mkdir -p $out
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "gemm and (72 or 100)" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "blocked_w" > $out/parity.log 2>&1 || { echo "parity failed"; tail -30 $out/parity.log; exit 1; }
  tail -2 $out/parity.log
  timeout -k 10 300 python -u tools/gemm_ab.py "10752,3072,768,1;2048,3072,768,1;12800,2304,768,0" \
    "3462,3472,13472,81,10081,98,10098" 5 20 > $out/ab.log 2>&1 || { echo "ab failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning w_blocked=1" \
    "--tuning w_blocked=1;split_variants=72,81" "--tuning w_blocked=1;split_variants=72,81;qkv_variant=3472" \
    > $out/inmodel.log 2>&1 || { echo "in-model A/B failed"; tail -20 $out/inmodel.log; exit 1; }
  cat $out/inmodel.log
}

run_yardstick() {
  out=gpurun_out/r05_yardstick
  mkdir -p $out
  timeout -k 10 300 python -u tools/blas_yardstick.py --out $out/blas.jsonl > $out/blas.log 2>&1 || { echo "blas failed"; tail -5 $out/blas.log; exit 1; }
  GEMM_AB_DTYPE=2 timeout -k 10 300 python -u tools/gemm_ab.py "12800,2304,768,0;12800,3072,768,0;10752,3072,768,0;12800,768,768,0;12800,768,3072,0;4096,4096,4096,0" "10098,10062,10072,10082,10008" 5 20 > $out/ours.log 2>&1 || { echo "ours failed"; tail -5 $out/ours.log; exit 1; }
  cat $out/blas.log $out/ours.log
}

[ $# -ge 1 ] || { sed -n "2,/^set -o/p" "$0" | sed "\$d"; exit 2; }
recipe=$1; shift
declare -F "run_$recipe" > /dev/null || { echo "unknown recipe: $recipe"; exit 2; }
"run_$recipe" "$@"
