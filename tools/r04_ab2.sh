#!/bin/bash
# r04 second session, GPU call 3: issue-slot ablations of the persistent tile (32x32x16 MFMA
# stand-ins, tools/exp_l2.sh), then the config-5 rocprof passes without the parity legs
LIBS="shipped nostage nomfma m32 m32nostage" VARS=62 bash tools/exp_l2.sh run > gpurun_out/exp_abl2.log 2>&1 || { cat gpurun_out/exp_abl2.log; exit 1; }
cat gpurun_out/exp_abl2.log
bash tools/profile_cfg5.sh gpurun_out/cfg5prof2 r04 && cat gpurun_out/cfg5prof2/summary.log
