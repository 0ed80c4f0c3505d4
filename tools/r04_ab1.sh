#!/bin/bash
# r04 second session, one GPU call:
#  1. bs-256 arms (same box, alternating): batches in flight, the two-lane split at bs 256 (shipped
#     tiles / CU-time-priced tiles), the c_fc main launch on the front-loaded persistent variants
#  2. tools/exp_l2.sh on the no-staging / no-MFMA ablation builds of the persistent tile
#  3. config-5 rocprof passes (tools/profile_cfg5.sh)
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--inflight 2" "--tuning split_min=256" \
  "--tuning split_min=256;gemm_variants=98,22,62,22,22;gemm_xcd=2,0,0,0,1" "--tuning split_variants=69,81" \
  "--tuning split_variants=70,81" || exit 1
LIBS="shipped nostage nomfma" VARS=62 bash tools/exp_l2.sh run > gpurun_out/exp_abl.log 2>&1 || { cat gpurun_out/exp_abl.log; exit 1; }
cat gpurun_out/exp_abl.log
bash tools/profile_cfg5.sh gpurun_out/cfg5prof r04 && cat gpurun_out/cfg5prof/summary.log
