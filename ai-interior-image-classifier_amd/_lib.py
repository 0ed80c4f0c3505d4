"""ctypes binding of libclipvit_hip.so (the C ABI in include/clipvit.h).

ctypes.CDLL releases the GIL around every foreign call, so concurrent ``encode``/``classify``
calls from host threads (the reference's ThreadPoolExecutor(4) pattern, main.py:345-346) run
in parallel inside the library. There is no fallback: if the library is missing or fails to
load, every entry point raises ``ClipVitError``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

# CLIPVIT_LIB: load another build of the library (same-box A/B of two builds, tools/ab_env.sh)
LIB_PATH = Path(os.environ.get("CLIPVIT_LIB") or Path(__file__).resolve().parent / "libclipvit_hip.so")

F32, BF16, F16, MXFP8 = 0, 1, 2, 3
OK, E_INVALID, E_HIP, E_STATE, E_NOMEM = 0, -1, -2, -3, -4

# Every symbol include/clipvit.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "clipvit_create", "clipvit_load_weights", "clipvit_load_lora", "clipvit_set_text_features",
    "clipvit_encode_image", "clipvit_classify", "clipvit_text_shape", "clipvit_destroy",
    "clipvit_last_error", "clipvit_abi_version", "clipvit_gemm_test", "clipvit_attention_test",
    "clipvit_profile_forward", "clipvit_gemm_bench", "clipvit_quant_mx8_test",
    "clipvit_gemm_mx8_test", "clipvit_preprocess", "clipvit_resample_plan",
    "clipvit_text_create", "clipvit_text_load_weights", "clipvit_text_load_lora",
    "clipvit_encode_text", "clipvit_text_destroy", "clipvit_residual_x24_test", "clipvit_set_tuning",
    "clipvit_gemm_log",
)


class ClipVitError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"clipvit error {code}: {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "image_size", "patch_size", "width", "layers", "heads", "embed_dim", "compute_dtype",
        "max_batch")]


class TextConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "width", "layers", "heads", "context", "vocab", "embed_dim", "compute_dtype", "max_batch")]


class Tensor(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.POINTER(ctypes.c_float)),
                ("ndim", ctypes.c_int), ("shape", ctypes.c_int64 * 4)]


class Image(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("width", ctypes.c_int), ("height", ctypes.c_int)]


class Lora(ctypes.Structure):
    _fields_ = [("target", ctypes.c_char_p), ("A", ctypes.POINTER(ctypes.c_float)),
                ("B", ctypes.POINTER(ctypes.c_float)), ("in_features", ctypes.c_int),
                ("out_features", ctypes.c_int), ("rank", ctypes.c_int), ("scaling", ctypes.c_float)]


_lock = threading.Lock()
_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the library; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise ClipVitError(E_STATE, f"{LIB_PATH} is not built (run __graft_entry__.build())")
        L = ctypes.CDLL(str(LIB_PATH))
        vp, i, p_f = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float)
        sig = {
            "clipvit_create": (i, [ctypes.POINTER(Config), i, ctypes.POINTER(vp)]),
            "clipvit_set_tuning": (i, [vp, ctypes.c_char_p]),
            "clipvit_load_weights": (i, [vp, ctypes.POINTER(Tensor), ctypes.c_size_t]),
            "clipvit_load_lora": (i, [vp, ctypes.POINTER(Lora), ctypes.c_size_t]),
            "clipvit_set_text_features": (i, [vp, p_f, i, i, ctypes.POINTER(ctypes.c_int), i]),
            "clipvit_encode_image": (i, [vp, vp, vp, i, i, vp]),
            "clipvit_classify": (i, [vp, vp, vp, i, i, vp, vp, vp, vp, vp]),
            "clipvit_text_shape": (i, [vp, ctypes.POINTER(i), ctypes.POINTER(i)]),
            "clipvit_destroy": (i, [vp]),
            "clipvit_last_error": (ctypes.c_char_p, []),
            "clipvit_abi_version": (i, []),
            "clipvit_gemm_test": (i, [vp, i, vp, vp, vp, vp, i, i, i, i, i]),
            "clipvit_attention_test": (i, [vp, i, vp, vp, i, i, i, i]),
            "clipvit_residual_x24_test": (i, [vp, vp, vp, vp, ctypes.c_size_t]),
            "clipvit_quant_mx8_test": (i, [vp, i, vp, i, i, vp, vp]),
            "clipvit_gemm_mx8_test": (i, [vp, vp, vp, vp, vp, vp, vp, i, i, i, i, i]),
            "clipvit_profile_forward": (i, [vp, vp, vp, i, i, i, p_f]),
            "clipvit_gemm_log": (i, [vp, ctypes.POINTER(i), i]),
            "clipvit_gemm_bench": (i, [i, i, i, i, i, i, i, p_f]),
            "clipvit_text_create": (i, [ctypes.POINTER(TextConfig), i, ctypes.POINTER(vp)]),
            "clipvit_text_load_weights": (i, [vp, ctypes.POINTER(Tensor), ctypes.c_size_t]),
            "clipvit_text_load_lora": (i, [vp, ctypes.POINTER(Lora), ctypes.c_size_t]),
            "clipvit_encode_text": (i, [vp, vp, vp, i, i, vp]),
            "clipvit_text_destroy": (i, [vp]),
            "clipvit_preprocess": (i, [vp, vp, ctypes.POINTER(Image), i, i, i, vp]),
            "clipvit_resample_plan": (i, [i, i, ctypes.POINTER(i), ctypes.POINTER(i),
                                          ctypes.POINTER(ctypes.c_int32), i]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
        return L


def check(rc: int) -> None:
    if rc != OK:
        msg = lib().clipvit_last_error()
        raise ClipVitError(rc, msg.decode("utf-8", "replace") if msg else "")
