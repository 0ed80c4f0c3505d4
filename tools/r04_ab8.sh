#!/bin/bash
# r04 closing session: class-token tail split-K rule (tuning tail_kmin / tail_smax), same box.
# First call: more slices (smax 12 / 16 / 48) made the tail slower (0.054-0.084 ms against 0.047);
# this call tries fewer.
set -o pipefail
bash tools/ab_envs.sh "" 2 - "--tuning tail_smax=4" "--tuning tail_smax=2" "--tuning tail_kmin=384"
