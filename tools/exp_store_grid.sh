#!/bin/bash
# store-epilogue A/B of the persistent ping-pong GEMM: shipped library vs the
# no-store ablation build (ab/nostore.so), variants 62 (stores from the accumulators) and 64
# (row-contiguous stores through LDS), two round counts so the per-tile slope separates from
# the per-launch cost. CLIPVIT_BENCH_GRID=g runs the persistent grid on g workgroups.
set -o pipefail
R=$(pwd)
SHAPES=${SHAPES:-"10752,3072,768,0;21504,3072,768,0;10752,3072,768,1;21504,3072,768,1"}
for lib in shipped nostore; do
  L=""; [ $lib = nostore ] && L=$R/ab/nostore.so
  for g in ${GRIDS:-256}; do
    echo "== $lib grid $g"
    CLIPVIT_LIB=$L CLIPVIT_BENCH_GRID=$g timeout -k 10 100 python tools/gemm_ab.py "$SHAPES" "${VARS:-64,62}" 3 10 || exit 1
  done
done
