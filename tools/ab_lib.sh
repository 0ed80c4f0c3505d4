#!/bin/bash
# GPU box: GPU tests on the in-tree build, then same-box A/B of ab/base.so (a previous build,
# copied there before rebuilding) against the in-tree library. Args: bench configs to A/B
# ("b32", "b16", "l14", "bf16", "mx"; default b32 b16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lib_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lib_t.log; exit 1; }
tail -1 gpurun_out/lib_t.log
NEW=$PWD/ai-interior-image-classifier_amd/libclipvit_hip.so; OLD=$PWD/ab/base.so
CFGS=${*:-b32 b16}
for c in $CFGS; do
  case $c in
    b32) bash tools/ab_env.sh "" CLIPVIT_LIB "$OLD $NEW" 3 || exit 1 ;;
    b16) bash tools/ab_env.sh "--model ViT-B/16" CLIPVIT_LIB "$OLD $NEW" 2 || exit 1 ;;
    l14) bash tools/ab_env.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" CLIPVIT_LIB "$OLD $NEW" 1 || exit 1 ;;
    bf16) bash tools/ab_env.sh "--dtype bf16 --batch 512" CLIPVIT_LIB "$OLD $NEW" 2 || exit 1 ;;
    mx) bash tools/ab_env.sh "--dtype mxfp8 --batch 512" CLIPVIT_LIB "$OLD $NEW" 2 || exit 1 ;;
  esac
done
