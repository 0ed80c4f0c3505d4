#!/bin/bash
# Host-side AddressSanitizer + UBSan build of libclipvit_hip.so and the ABI stress driver
# (tools/asan/abi_stress.cpp). Only host code is instrumented (-Xarch_host puts each
# -fsanitize= on the host compile); the gfx950 device code is unchanged. Outputs go to
# tools/asan/out/ (git-ignored). Run on the GPU box:
#   ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=1 tools/asan/out/abi_stress
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/tools/asan/out
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$ROOT/ai-interior-image-classifier_amd/csrc -mllvm --amdgpu-mfma-vgpr-form -Wno-unused-result -Wno-unused-value"
objs=""
for src in "$ROOT"/ai-interior-image-classifier_amd/csrc/*.hip; do
  o=$OUT/$(basename "$src" .hip).o
  $HIPCC $FLAGS $SAN -c "$src" -o "$o" &
  objs="$objs $o"
done
wait
$HIPCC --offload-arch=gfx950 -shared -fno-gpu-sanitize -fsanitize=address -fsanitize=undefined -o "$OUT/libclipvit_asan.so" $objs
$HIPCC $FLAGS $SAN -x hip "$ROOT/tools/asan/abi_stress.cpp" -o "$OUT/abi_stress" \
  -L"$OUT" -lclipvit_asan -Wl,-rpath,"\$ORIGIN" -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined
echo "built $OUT/abi_stress"
