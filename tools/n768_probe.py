"""Tile probe for the N = 768 roles (out_proj, c_proj, patch) at B/32 bs 256 (GPU box).

    python tools/n768_probe.py
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from split_probe import t  # noqa: E402

for name, M, K, epi, vs in [("out", 12800, 768, 0, [282, 82, 92, 292, 94, 294]),
                            ("proj", 12800, 3072, 0, [282, 82, 92, 292, 94, 294]),
                            ("patch", 12544, 3072, 3, [122, 22, 93, 293, 95, 295])]:
    for v in vs:
        us = t(M, 768, K, epi, v)
        print(f"{name} v{v}: {us:.1f} us  {2*M*768*K/us/1e6:.0f} TF/s", flush=True)
