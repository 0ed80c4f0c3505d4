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

recipe=${1:-}
shift || true
case "$recipe" in
  check) run_check "$@" ;;
  tests) run_tests "$@" ;;
  ab) run_ab "$@" ;;
  *) echo "recipes: check | tests <expr> [files] | ab '<bench args>' R arm..."; exit 2 ;;
esac
