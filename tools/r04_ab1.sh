#!/bin/bash
# r04 second session, one GPU call: bs-256 arms (same box, alternating) — batches in flight, the
# two-lane split at bs 256 (shipped tiles / CU-time-priced tiles), and the c_fc main launch on the
# front-loaded persistent variants 69 / 70
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--inflight 2" "--tuning split_min=256" \
  "--tuning split_min=256;gemm_variants=98,22,62,22,22;gemm_xcd=2,0,0,0,1" "--tuning split_variants=69,81" \
  "--tuning split_variants=70,81"
