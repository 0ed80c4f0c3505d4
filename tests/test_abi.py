"""The C-ABI library loads and exports every symbol include/clipvit.h declares (CPU only:
no compute calls; on a host without a GPU, create must fail with a status, not crash)."""
import ctypes
import re
from pathlib import Path

import pytest
import torch

from interior_amd import _lib

HEADER = Path(__file__).resolve().parents[1] / "include" / "clipvit.h"


def declared_symbols():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(clipvit_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("clipvit_create", "clipvit_load_weights", "clipvit_load_lora",
              "clipvit_set_text_features", "clipvit_encode_image", "clipvit_classify",
              "clipvit_destroy", "clipvit_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_abi_version():
    assert _lib.lib().clipvit_abi_version() == 4  # 3: clipvit_set_tuning (no environment reads); 4: clipvit_gemm_log


def test_struct_layouts_match_header():
    # clipvit_config: 8 ints; clipvit_tensor: ptr, ptr, int (+pad), 4 x int64; clipvit_lora
    assert ctypes.sizeof(_lib.Config) == 32
    assert ctypes.sizeof(_lib.Tensor) == 8 + 8 + 8 + 32
    assert ctypes.sizeof(_lib.Lora) == 8 * 3 + 4 * 4


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU error path")
def test_create_without_gpu_reports_error():
    L = _lib.lib()
    cfg = _lib.Config(224, 32, 768, 12, 12, 512, _lib.F16, 4)
    h = ctypes.c_void_p()
    rc = L.clipvit_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc != 0 and L.clipvit_last_error()


def test_invalid_config_rejected_before_device_work():
    L = _lib.lib()
    h = ctypes.c_void_p()
    bad = _lib.Config(224, 32, 768, 12, 11, 512, _lib.F16, 4)  # heads * 64 != width
    assert L.clipvit_create(ctypes.byref(bad), 0, ctypes.byref(h)) == _lib.E_INVALID
    assert b"heads" in L.clipvit_last_error()


def test_engine_refuses_cpu():
    from interior_amd.config import VIT_B32
    from interior_amd.engine import VisionEngine
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.ClipVitError):
        VisionEngine(VIT_B32, 0)
