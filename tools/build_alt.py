"""Build an A/B variant of libclipvit_hip.so with extra preprocessor defines (CPU side).

    python tools/build_alt.py NAME UNIT[,UNIT...] -DKEY=VALUE ...

Recompiles only the listed translation units (csrc/<UNIT>.hip) with the defines into alt/NAME/,
links them with the default build's other objects and writes alt/NAME.so (git-ignored but not
gpurun-ignored: the .so travels to the GPU box). Compare on one box with tools/ab_envs.sh arms
"CLIPVIT_LIB=$PWD/alt/NAME.so".
"""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import build as b  # noqa: E402

name, units, defs = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
out = b.ROOT / "alt" / name
out.mkdir(parents=True, exist_ok=True)
b.build()
objs = []
for src in b._sources():
    if src.stem in units:
        obj = out / (src.stem + ".o")
        cmd = [b.HIPCC, *b.CFLAGS, *b.SRC_FLAGS.get(src.stem, []), *defs, "-c", str(src), "-o", str(obj)]
        subprocess.run(cmd, check=True)
        objs.append(obj)
    else:
        objs.append(b.BUILD / (src.stem + ".o"))
lib = b.ROOT / "alt" / f"{name}.so"
subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-o", str(lib), *map(str, objs)], check=True)
print(lib)
