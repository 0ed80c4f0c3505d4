#!/bin/bash
# Round-6 GPU recipes (one function per measurement; outputs under gpurun_out/r06_*, the kept
# ones copied to profiles/r06/). Run from the repo root, on the GPU box:
#   bash tools/r06_runs.sh <recipe> [args]
# Every GPU step runs under its own time limit; the first failure ends the call.
set -o pipefail

# full GPU suite + smoke + the default bench line + the self-launched 2-rank rehearsal
run_check() {
  out=gpurun_out/r06_check
  mkdir -p $out
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs \
    > $out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/gpu_tests.log; exit 1; }
  tail -3 $out/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
  timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['family_ms_per_forward'])"
}

# a subset of the GPU tests by -k expression: bash tools/r06_runs.sh tests "<expr>" [file...]
run_tests() {
  out=gpurun_out/r06_tests
  mkdir -p $out
  expr=$1; shift
  files=${*:-tests}
  timeout -k 10 600 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread -s -k "$expr" \
    > $out/tests.log 2>&1 || { echo "tests failed"; tail -60 $out/tests.log; exit 1; }
  grep -E "PASSED|FAILED|SKIPPED|passed|failed" $out/tests.log | tail -40
}

# same-box A/B of bench arms (tools/ab_envs.sh): bash tools/r06_runs.sh ab "<bench args>" R arm...
run_ab() {
  out=gpurun_out/r06_ab
  mkdir -p $out
  args=$1; R=$2; shift 2
  timeout -k 10 1000 bash tools/ab_envs.sh "$args" "$R" "$@" > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
}

# variant 77 (320 x 256 balanced c_fc tile): kernel tests, kernel A/B against v75, in-model A/B
run_t320() {
  out=gpurun_out/r06_t320
  mkdir -p $out
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "77 or race" > $out/kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 $out/kernels.log; exit 1; }
  tail -2 $out/kernels.log
  timeout -k 10 300 python -u tools/gemm_ab.py "12800,3072,768,1;12800,2304,768,0" "13475,13477,3475,3477,98,13472" 5 20 \
    > $out/gemm_ab.log 2>&1 || { echo "gemm_ab failed"; tail -10 $out/gemm_ab.log; exit 1; }
  cat $out/gemm_ab.log
  timeout -k 10 900 bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning fc_balanced_variant=77" > $out/ab.log 2>&1 \
    || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
}

# The GEMM k-loop split into phases: the stamped shipped kernel (gemm_probe
# p32, hook policy P32Stamp) on the c_fc shape as shipped (balanced grid, map 34) and on the QKV
# shape, the ablations, then per-role PMC passes of the default bench (LDS / VMEM issue, TA, TCP).
run_phases() {
  R=$GRAFT_REPO_ROOT
  out=$R/gpurun_out/r06_phases
  mkdir -p $out
  P=$R/tools/probes/gemm_probe
  { echo "== c_fc 12800x3072x768 gelu xcd34 balanced"; timeout -k 10 120 $P p32 12800 3072 768 1 34 1 && \
    echo "== QKV 12800x2304x768 store xcd0"; timeout -k 10 120 $P p32 12800 2304 768 0 0 0; } > $out/stamps.txt 2>&1 \
    || { echo "probe failed"; tail -20 $out/stamps.txt; exit 1; }
  cat $out/stamps.txt
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || echo "counter list failed"
  grep -oE "(TA_[A-Z_]+|TCP_PENDING[A-Z_]*|SQ_INST_CYCLES_VMEM|SQ_WAIT_INST_LDS|SQ_INSTS_LDS)" $out/counters.txt | sort -u | head -40 || true
  B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --profile-iters 1"
  i=0
  for set in "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
             "TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $out/pmc$i -o run -- $B > $out/pmc$i.log 2>&1 \
      || { rc=$?; echo "pass $i ($set) failed rc=$rc"; tail -3 $out/pmc$i.log; [ $rc -ge 124 ] && exit 1; }
  done
  echo phases-done
}

# blocked A (h in the 16-row blocked layout): kernel bit-identity, then kernel A/B on the B/32
# c_fc (v75) and QKV (v98) shapes, row-major A against blocked A (both with blocked W)
run_ablk() {
  out=gpurun_out/r06_ablk
  mkdir -p $out
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "blocked_a" > $out/kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 $out/kernels.log; exit 1; }
  tail -2 $out/kernels.log
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "blocked_h" > $out/parity.log 2>&1 || { echo "parity tests failed"; tail -30 $out/parity.log; exit 1; }
  tail -2 $out/parity.log
  timeout -k 10 900 bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning h_blocked=1" "--tuning h_blocked=2" > $out/ab.log 2>&1 \
    || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
  cat $out/ab.log
}

# kernel-level tile sweep of the N = 768 roles and QKV at B/32 bs 256 (blocked W; c_proj's A is the
# blocked u: + 30000)
run_tiles() {
  out=gpurun_out/r06_tiles
  mkdir -p $out
  timeout -k 10 600 python -u tools/gemm_ab.py "12800,768,768,0" "10082,10081,10022,10080,10098,10008,13472,13475,13462" 5 20 \
    > $out/out.log 2>&1 || { echo "out_proj sweep failed"; tail -10 $out/out.log; exit 1; }
  cat $out/out.log
  timeout -k 10 600 python -u tools/gemm_ab.py "12800,768,3072,0" "30082,30081,30022,30080,30098,33472,33475,33462" 5 20 \
    > $out/proj.log 2>&1 || { echo "c_proj sweep failed"; tail -10 $out/proj.log; exit 1; }
  cat $out/proj.log
  timeout -k 10 600 python -u tools/gemm_ab.py "12800,2304,768,0" "10298,10098,10082,10022,13472,13475,13462,10080" 5 20 \
    > $out/qkv.log 2>&1 || { echo "qkv sweep failed"; tail -10 $out/qkv.log; exit 1; }
  cat $out/qkv.log
}

# the round's profile (tools/profile_round.sh: kernel trace + FETCH / WRITE / MFMA / L2 passes,
# then the default bench with its PMC traffic) and the other configurations' bench lines
run_closing() {
  tag=${1:-r06}
  out=gpurun_out/${tag}_closing
  mkdir -p $out
  timeout -k 10 1100 bash tools/profile_round.sh gpurun_out/prof_$tag $tag > $out/profile.log 2>&1 \
    || { echo "profile round failed"; tail -20 $out/profile.log; exit 1; }
  tail -2 $out/profile.log
  for c in "cfg4|--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" \
           "b16|--model ViT-B/16 --steps 10 --warmup 3" \
           "b32_bf16|--dtype bf16 --steps 20 --warmup 5" \
           "cfg5_mx|--dtype mxfp8 --batch 512 --steps 20 --warmup 5" \
           "cfg5_bf16|--dtype bf16 --batch 512 --steps 20 --warmup 5 --no-cpu-baseline"; do
    name=${c%%|*}; args=${c#*|}
    timeout -k 10 300 python bench.py $args > $out/$name.json 2> $out/$name.err \
      || { echo "bench $name failed"; tail -10 $out/$name.err; exit 1; }
    python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('parity'))"
  done
}

recipe=${1:-}
shift || true
case "$recipe" in
  check) run_check "$@" ;;
  tests) run_tests "$@" ;;
  ab) run_ab "$@" ;;
  t320) run_t320 "$@" ;;
  phases) run_phases "$@" ;;
  ablk) run_ablk "$@" ;;
  tiles) run_tiles "$@" ;;
  closing) run_closing "$@" ;;
  *) echo "recipes: check | tests <expr> [files] | ab '<bench args>' R arm..."; exit 2 ;;
esac
