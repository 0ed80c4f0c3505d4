"""VisionEngine: one C-ABI handle (one GPU) running the CLIP-ViT image path.

PyTorch is plumbing here: it owns device buffers and streams; every FLOP of the encoder and
head runs in libclipvit_hip.so's hand-written gfx950 kernels. There is no CPU fallback: without
the library or without a GPU the constructor raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .config import ViTConfig
from .lora import LoraAdapter
from .weights import as_host_f32, visual_names

_DT = {"bf16": _lib.BF16, "fp16": _lib.F16, "f16": _lib.F16, torch.bfloat16: _lib.BF16,
       torch.float16: _lib.F16, "mxfp8": _lib.MXFP8}
_PIX_DT = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float16: _lib.F16}


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _vp(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


@dataclass
class ClassifyOutput:
    emb: torch.Tensor        # [B, E] L2-normalised features
    logits: torch.Tensor     # [B, C] 100 * cos
    probs: torch.Tensor      # [B, C] softmax within each segment
    top_idx: torch.Tensor    # [B, nseg, 5] int32, index inside the segment (-1 padding)
    top_prob: torch.Tensor   # [B, nseg, 5]


class VisionEngine:
    def __init__(self, cfg: ViTConfig, device: int | str | torch.device = 0,
                 compute_dtype: str = "fp16", max_batch: int = 256, tuning: dict | str | None = None):
        """``tuning``: tests and A/B tools only — one of DESIGN.md's measured alternatives
        instead of the shipped default (clipvit_set_tuning; e.g. ``{"split_min": 0}``)."""
        if not torch.cuda.is_available():
            raise _lib.ClipVitError(_lib.E_STATE, "no HIP device visible: the MI355X path needs a GPU")
        dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
        if dev.type != "cuda":
            raise ValueError("VisionEngine runs on a HIP device ('cuda:N' in PyTorch-ROCm)")
        self.device = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        self.cfg = cfg
        self.compute_dtype = compute_dtype
        self.max_batch = int(max_batch)
        self._L = _lib.lib()
        c = _lib.Config(cfg.image_size, cfg.patch_size, cfg.width, cfg.layers, cfg.heads,
                        cfg.embed_dim, _DT[compute_dtype], self.max_batch)
        h = ctypes.c_void_p()
        _lib.check(self._L.clipvit_create(ctypes.byref(c), self.device.index, ctypes.byref(h)))
        self._h = h
        if tuning:
            spec = tuning if isinstance(tuning, str) else ";".join(f"{k}={v}" for k, v in tuning.items())
            try:
                _lib.check(self._L.clipvit_set_tuning(h, spec.encode()))
            except Exception:
                self.close()
                raise
        self.tuning = tuning
        self.C = 0
        self.seg_offsets: list[int] = []
        self.loaded = False

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self._L.clipvit_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- weights
    def load_state_dict(self, sd: dict) -> None:
        """``visual.*`` tensors (OpenAI names, any float dtype) -> HBM (clipvit_load_weights)."""
        names = visual_names(self.cfg)
        keep, arr = [], (_lib.Tensor * len(names))()
        for i, (name, shape) in enumerate(names):
            if name not in sd:
                raise KeyError(f"missing {name}")
            a = as_host_f32(sd[name])
            if tuple(a.shape) != tuple(shape):
                raise ValueError(f"{name}: shape {a.shape} != {shape}")
            keep.append(a)
            bn = name.encode()
            keep.append(bn)
            arr[i].name = bn
            arr[i].data = _fptr(a)
            arr[i].ndim = a.ndim
            for d in range(a.ndim):
                arr[i].shape[d] = a.shape[d]
        _lib.check(self._L.clipvit_load_weights(self._h, arr, len(names)))
        self.loaded = True

    def load_lora(self, adapters: list[LoraAdapter]) -> None:
        """Merge adapters into the vision Linears (replaces any previously merged set)."""
        keep, arr = [], (_lib.Lora * max(len(adapters), 1))()
        for i, ad in enumerate(adapters):
            A, B = as_host_f32(ad.A), as_host_f32(ad.B)
            t = ad.target.encode()
            keep += [A, B, t]
            arr[i].target, arr[i].A, arr[i].B = t, _fptr(A), _fptr(B)
            arr[i].in_features, arr[i].out_features = A.shape[0], B.shape[1]
            arr[i].rank, arr[i].scaling = A.shape[1], float(ad.scaling)
        _lib.check(self._L.clipvit_load_lora(self._h, arr, len(adapters)))

    def set_text_features(self, T, seg_offsets: list[int]) -> None:
        """T [C, E] L2-normalised text features; segments = label groups (detector, styles...)."""
        T = as_host_f32(T)
        off = (ctypes.c_int * len(seg_offsets))(*seg_offsets)
        _lib.check(self._L.clipvit_set_text_features(self._h, _fptr(T), T.shape[0], T.shape[1], off,
                                                     len(seg_offsets) - 1))
        self.C = T.shape[0]
        self.seg_offsets = list(seg_offsets)

    # ---------------------------------------------------------------- compute
    def _pixels(self, pixels: torch.Tensor) -> torch.Tensor:
        R = self.cfg.image_size
        if pixels.dim() != 4 or tuple(pixels.shape[1:]) != (3, R, R):
            raise ValueError(f"pixels must be [B, 3, {R}, {R}], got {tuple(pixels.shape)}")
        if pixels.shape[0] == 0:
            raise _lib.ClipVitError(_lib.E_INVALID, "empty batch")
        if pixels.dtype not in _PIX_DT:
            pixels = pixels.float()
        if pixels.device != self.device:
            pixels = pixels.to(self.device, non_blocking=True)
        return pixels.contiguous()

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def encode_image(self, pixels: torch.Tensor) -> torch.Tensor:
        """model.encode_image (main.py:204/444/503): [B,3,R,R] -> [B,E] fp32 on the device."""
        if not self.loaded:
            raise _lib.ClipVitError(_lib.E_STATE, "weights not loaded")
        pixels = self._pixels(pixels)
        B = pixels.shape[0]
        out = torch.empty((B, self.cfg.embed_dim), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            s = self._stream()
            for a in range(0, B, self.max_batch):
                b = min(B, a + self.max_batch)
                _lib.check(self._L.clipvit_encode_image(self._h, s, _vp(pixels[a:b]),
                                                        _PIX_DT[pixels.dtype], b - a, _vp(out[a:b])))
        return out

    def classify(self, pixels: torch.Tensor, out: ClassifyOutput | None = None) -> ClassifyOutput:
        """encode_image + L2-norm + 100*cos logits + per-segment softmax/top-5, on device."""
        if not self.loaded or not self.C:
            raise _lib.ClipVitError(_lib.E_STATE, "weights or text features not set")
        pixels = self._pixels(pixels)
        B = pixels.shape[0]
        nseg = len(self.seg_offsets) - 1
        if out is None:
            kw = dict(device=self.device)
            out = ClassifyOutput(
                emb=torch.empty((B, self.cfg.embed_dim), dtype=torch.float32, **kw),
                logits=torch.empty((B, self.C), dtype=torch.float32, **kw),
                probs=torch.empty((B, self.C), dtype=torch.float32, **kw),
                top_idx=torch.empty((B, nseg, 5), dtype=torch.int32, **kw),
                top_prob=torch.empty((B, nseg, 5), dtype=torch.float32, **kw))
        with torch.cuda.device(self.device):
            s = self._stream()
            for a in range(0, B, self.max_batch):
                b = min(B, a + self.max_batch)
                _lib.check(self._L.clipvit_classify(
                    self._h, s, _vp(pixels[a:b]), _PIX_DT[pixels.dtype], b - a, _vp(out.emb[a:b]),
                    _vp(out.logits[a:b]), _vp(out.probs[a:b]), _vp(out.top_idx[a:b]),
                    _vp(out.top_prob[a:b])))
        return out

    def profile_forward(self, pixels: torch.Tensor, iters: int = 5) -> dict[str, float]:
        """Per-kernel-family device milliseconds of one forward (HIP events between stages)."""
        pixels = self._pixels(pixels)
        ms = (ctypes.c_float * 20)()
        with torch.cuda.device(self.device):
            _lib.check(self._L.clipvit_profile_forward(self._h, self._stream(), _vp(pixels),
                                                       _PIX_DT[pixels.dtype], pixels.shape[0], iters, ms))
        fams = ("patch_embed", "qkv_gemm", "attention", "out_proj_gemm", "layernorm", "fc_gemm",
                "proj_gemm", "head", "cls_tail")
        out = {k: float(v) for k, v in zip(fams, ms)}
        out["lane_batch"] = float(ms[9])
        out["intervals"] = {k: int(ms[10 + i]) for i, k in enumerate(fams)}
        out["event_gap_ms"] = float(ms[19])
        return out

    def gemm_log(self, cap: int = 4096) -> list[tuple[int, int, int, int]]:
        """Test hook: the (role, tile variant, M, flags) of every Linear-role GEMM launch since the
        last call (needs tuning trace_gemm=1; clipvit_gemm_log). Roles: 0 qkv, 1 out_proj, 2 c_fc,
        3 c_proj; flags: 1 blocked W copy, 2 MX-fp8, 4 blocked A, 8 blocked C."""
        buf = (ctypes.c_int * (4 * cap))()
        n = self._L.clipvit_gemm_log(self._h, buf, cap)
        if n < 0:
            _lib.check(n)
        return [tuple(buf[4 * i:4 * i + 4]) for i in range(n)]


# ------------------------------------------------------------------ kernel-level helpers
def gemm_test(A: torch.Tensor, W: torch.Tensor, bias: torch.Tensor | None, epi: int = 0,
              variant: int = 0, C: torch.Tensor | None = None) -> torch.Tensor:
    """C = A @ W^T + bias through the library's MFMA GEMM (A bf16/f16 on device, W fp32)."""
    L = _lib.lib()
    M, K = A.shape
    N = W.shape[0]
    if C is None:
        C = torch.zeros((M, N), dtype=torch.float32, device=A.device)
    W32 = W.float().contiguous()  # held until the stream-ordered pack kernel has read it
    with torch.cuda.device(A.device):
        s = ctypes.c_void_p(torch.cuda.current_stream(A.device).cuda_stream)
        _lib.check(L.clipvit_gemm_test(s, _DT[A.dtype], _vp(A), _vp(W32), _vp(bias), _vp(C), M, N,
                                       K, epi, variant))
        torch.cuda.current_stream(A.device).synchronize()
    return C


def quant_mx8_test(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """MX-fp8 quantization of a [rows, K] fp32/bf16/fp16 device tensor by the library's
    kernel: (e4m3 bytes [rows, K] uint8, E8M0 scales [rows, K/32] uint8)."""
    L = _lib.lib()
    x = x.contiguous()
    rows, K = x.shape
    q = torch.empty((rows, K), dtype=torch.uint8, device=x.device)
    sq = torch.empty((rows, K // 32), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _lib.check(L.clipvit_quant_mx8_test(s, _PIX_DT[x.dtype], _vp(x), rows, K, _vp(q), _vp(sq)))
        torch.cuda.current_stream(x.device).synchronize()
    return q, sq


def gemm_mx8_test(A8: torch.Tensor, sA: torch.Tensor, W: torch.Tensor, bias: torch.Tensor | None,
                  epi: int = 0, variant: int = 0, C: torch.Tensor | None = None):
    """MX-fp8 GEMM through the library (clipvit_gemm_mx8_test). epi 0/1/2 -> fp32 C,
    3/4 -> (C uint8 [M,N], sC uint8 [M,N/32]), 5 -> bf16 C."""
    L = _lib.lib()
    M, K = A8.shape
    N = W.shape[0]
    dev = A8.device
    sC = None
    if C is None:
        if epi in (0, 1, 2):
            C = torch.zeros((M, N), dtype=torch.float32, device=dev)
        elif epi in (3, 4):
            C = torch.zeros((M, N), dtype=torch.uint8, device=dev)
        else:
            C = torch.zeros((M, N), dtype=torch.bfloat16, device=dev)
    if epi in (3, 4):
        sC = torch.zeros((M, N // 32), dtype=torch.uint8, device=dev)
    W32 = W.float().contiguous()
    with torch.cuda.device(dev):
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(L.clipvit_gemm_mx8_test(s, _vp(A8), _vp(sA), _vp(W32), _vp(bias), _vp(C), _vp(sC),
                                           M, N, K, epi, variant))
        torch.cuda.current_stream(dev).synchronize()
    return (C, sC) if epi in (3, 4) else C


def residual_x24_test(x: torch.Tensor) -> torch.Tensor:
    """fp32 x (numel % 4 == 0) through the 24-bit residual planes and back (norm.hip x24_store /
    x24_load)."""
    L = _lib.lib()
    x = x.contiguous()
    planes = torch.empty(x.numel() * 3, dtype=torch.uint8, device=x.device)
    back = torch.empty_like(x)
    with torch.cuda.device(x.device):
        s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _lib.check(L.clipvit_residual_x24_test(s, _vp(x), _vp(planes), _vp(back), x.numel()))
    return back


def attention_test(qkv: torch.Tensor, B: int, N: int, H: int, causal: bool = False, persist: int = 0) -> torch.Tensor:
    """clipvit_attention_test; persist > 0 (N <= 64): the persistent one-key-block kernel on that
    many workgroups per CU (tuning attn_persist)."""
    L = _lib.lib()
    out = torch.empty((B * N, H * 64), dtype=qkv.dtype, device=qkv.device)
    with torch.cuda.device(qkv.device):
        s = ctypes.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
        _lib.check(L.clipvit_attention_test(s, _DT[qkv.dtype], _vp(qkv), _vp(out), B, N, H, int(causal) | (persist << 4)))
    return out
