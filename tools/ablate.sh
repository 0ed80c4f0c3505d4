#!/bin/bash
# Diagnostic builds of the library (CPU side, this container): ab/noload.so (GEMM operand fill
# removed: MFMAs on stale LDS) and ab/nomfma.so (GEMM MFMAs removed: fill, barriers and
# epilogue only). Outputs are garbage; only the GEMM family times mean anything. Compare with
# tools/ab_envs.sh "<args>" R - CLIPVIT_LIB=$PWD/ab/noload.so CLIPVIT_LIB=$PWD/ab/nomfma.so
# (CLIPVIT_ABLATE=3, no epilogue stores in the persistent ping-pong GEMM, is built the same way
# for gemm_pp.hip alone: DESIGN.md §5.8.)
set -e
cd "$(dirname "$0")/.."
mkdir -p ab/abl1 ab/abl2
for v in 1 2; do
  for f in ai-interior-image-classifier_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Iai-interior-image-classifier_amd/csrc \
      -mllvm --amdgpu-mfma-vgpr-form -Wno-unused-result -Wno-unused-value -DCLIPVIT_ABLATE=$v \
      -c "$f" -o "ab/abl$v/$(basename "$f" .hip).o" &
  done
  wait
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ab/noload.so ab/abl1/*.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ab/nomfma.so ab/abl2/*.o
echo ablate-built
