"""In-tree build of libclipvit_hip.so (gfx950 only).

Compiles every ``csrc/*.hip`` translation unit with ``hipcc --offload-arch=gfx950`` in
parallel and links them into ``libclipvit_hip.so`` next to this file, so the shared library
travels with the repository snapshot to the GPU box. Incremental: a unit is recompiled only
when it, a ``csrc/*.h`` header or ``include/clipvit.h`` is newer than its object file.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
INCLUDE = ROOT / "include"
BUILD = PKG_DIR / "build"
LIB = PKG_DIR / "libclipvit_hip.so"
ARCH = "gfx950"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# --amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs. Without it the backend put the
# accumulators of tiles whose occupancy allows > 256 registers (the class-token tail's 2-wave
# 64x64 tile) in AGPRs and rotated them with v_accvgpr_mov/read/write every k-step.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}",
          "-mllvm", "--amdgpu-mfma-vgpr-form", "-Wno-unused-result", "-Wno-unused-value"]
# Per-source flags. gemm.hip: the max-memory-clause machine scheduler (clusters each k-step's
# staging loads). Same-box A/B of the two builds (profiles/design_r05.md §11): B/32 +0.2 / +0.6 %, B/16
# +0.5 %, L/14@336 +0.7 / +1.0 % img/s, patch GEMM -7 %; on attention.hip it cost 6 %, so
# only the GEMMs get it.
SRC_FLAGS = {"gemm": ["-mllvm", "--amdgpu-sched-strategy=max-memory-clause"]}
# options a unit is built without (none since the r05 one-wave-per-SIMD probes left the build)
SRC_DROP: dict[str, list[str]] = {}


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _needs(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _compile(src: Path) -> tuple[Path, str]:
    obj = BUILD / (src.stem + ".o")
    deps = [src, *CSRC.glob("*.h"), INCLUDE / "clipvit.h", Path(__file__)]  # this file: the flags
    if not _needs(obj, deps):
        return obj, ""
    flags = list(CFLAGS)
    for f in SRC_DROP.get(src.stem, []):  # a dropped -mllvm option takes its -mllvm with it
        i = flags.index(f)
        del flags[i - 1:i + 1]
    cmd = [HIPCC, *flags, *SRC_FLAGS.get(src.stem, []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile and link libclipvit_hip.so; return its path."""
    BUILD.mkdir(exist_ok=True)
    srcs = _sources()
    if force:
        for o in BUILD.glob("*.o"):
            o.unlink()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 16)
    with ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        results = list(ex.map(_compile, srcs))
    objs = [o for o, _ in results]
    if verbose:
        for o, err in results:
            if err.strip():
                print(f"[{o.name}] {err}", file=sys.stderr)
    if force or _needs(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
