#!/bin/bash
# Where the persistent ping-pong GEMM's k-tiles lose time at full chip:
# the shipped kernel against diagnostic builds of gemm_pp.hip in which every tile stages the
# same A panel (abx/l2a.so), the same W panel (abx/l2w.so) or both (abx/l2aw.so) — operands that
# then stay L2-resident — and in which the k-loop stages nothing after the first two k-tiles
# (abx/nostage.so), issues no MFMA (abx/nomfma.so, fragment reads kept), or issues one 32x32x16 MFMA
# per pair of 16x16x32 (abx/m32.so, abx/m32nostage.so: half the MFMA issue slots), at several persistent
# grid sizes (CLIPVIT_BENCH_GRID).
#   bash tools/exp_l2.sh build     (CPU, this container: the three libraries)
#   bash tools/exp_l2.sh run       (GPU: gemm_ab.py per library and grid)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/ai-interior-image-classifier_amd/build
if [ "$1" = build ]; then
  mkdir -p "$R/abx"
  for v in 4 5 6 7 8 9 10; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I"$R/include" -I"$R/ai-interior-image-classifier_amd/csrc" \
      -mllvm --amdgpu-mfma-vgpr-form -Wno-unused-result -Wno-unused-value -DCLIPVIT_ABLATE=$v \
      -c "$R/ai-interior-image-classifier_amd/csrc/gemm_pp.hip" -o "$R/abx/gemm_pp_$v.o" &
  done
  wait
  for v in 4 5 6 7 8 9 10; do
    case $v in 4) n=l2aw ;; 5) n=l2a ;; 6) n=l2w ;; 7) n=nostage ;; 8) n=nomfma ;; 9) n=m32 ;; 10) n=m32nostage ;; esac
    objs=$(ls "$B"/*.o | grep -v gemm_pp.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$R/abx/$n.so" $objs "$R/abx/gemm_pp_$v.o" || exit 1
  done
  echo exp_l2-built
  exit 0
fi
SHAPES=${SHAPES:-"10752,3072,768,1;12800,2304,768,0"}
for lib in ${LIBS:-shipped nostage nomfma m32 m32nostage}; do
  L=""; [ $lib != shipped ] && L=$R/abx/$lib.so
  for g in ${GRIDS:-256 64}; do
    echo "== $lib grid $g"
    V=${VARS:-62}
    CLIPVIT_LIB=$L CLIPVIT_BENCH_GRID=$g timeout -k 10 100 python tools/gemm_ab.py "$SHAPES" "$V" 3 10 || exit 1
  done
done
