#!/bin/bash
# r05: probe builds of gemm_w4.hip's schedule knobs (CPU side: builds abw4/*.so; GPU side with --run)
set -o pipefail
cd "$(dirname "$0")/.."
B=ai-interior-image-classifier_amd/build
if [ "$1" != "--run" ]; then
  mkdir -p abw4
  others=$(ls $B/*.o | grep -v gemm_w4.o)
  for cfg in "base:" "front:-DW4_FRONT=1" "front_noprio:-DW4_FRONT=1 -DW4_PRIO=0" "noprio:-DW4_PRIO=0"; do
    n=${cfg%%:*}; f=${cfg#*:}
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Iai-interior-image-classifier_amd/csrc \
      -Wno-unused-result -Wno-unused-value $f -c ai-interior-image-classifier_amd/csrc/gemm_w4.hip -o /tmp/w4_$n.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abw4/$n.so $others /tmp/w4_$n.o || exit 1
  done
  ls -la abw4
  exit 0
fi
out=gpurun_out/r05_w4_knobs
mkdir -p $out
for n in base front front_noprio noprio; do
  CLIPVIT_LIB=$PWD/abw4/$n.so GEMM_AB_DTYPE=2 timeout -k 10 300 python -u tools/gemm_ab.py "12800,2304,768,0;10752,3072,768,1;4096,4096,4096,0" "10076,10072" 5 20 > $out/$n.log 2>&1 || { echo "$n failed"; tail -5 $out/$n.log; exit 1; }
  echo "== $n"; cat $out/$n.log
done
