#!/bin/bash
# 256x256 MX-fp8 tiles (variants 3, 4) vs the 128x256 / 128x128 defaults (1, 2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mx8_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/mx8_tests.log | head; tail -3 gpurun_out/mx8_tests.log; exit 1; }
tail -1 gpurun_out/mx8_tests.log
timeout -k 10 200 python -u - <<'PY' > gpurun_out/mx8_tune.log 2>&1 || { tail gpurun_out/mx8_tune.log; exit 1; }
import ctypes, sys
sys.path.insert(0, ".")
import amd_pkg; amd_pkg.load()
import torch; torch.cuda.init()
from interior_amd import _lib
L = _lib.lib()
M = 512 * 50
for name, n, k, epi in (("qkv", 2304, 768, 0), ("out", 768, 768, 2), ("fc", 3072, 768, 1), ("proj", 768, 3072, 2)):
    for v in (201, 202, 203, 204, 1, 2, 3, 4):
        ms = ctypes.c_float()
        rc = L.clipvit_gemm_bench(3, M, n, k, epi, v, 30, ctypes.byref(ms))
        tf = 2.0 * M * n * k / (ms.value * 1e-3) / 1e12 if not rc else 0
        print(f"{name} v{v}: " + ("unsupported" if rc else f"{ms.value*1e3:.1f} us {tf:.0f} TF/s"), flush=True)
PY
cat gpurun_out/mx8_tune.log | grep -v amdgpu.ids
