"""L2 -> LDS fill bytes and implied rates of the GEMM roles (numbers for DESIGN.md 5.4).

    python tools/fill_model.py   (CPU; the times are the ablation builds' family ms per forward,
                                  tools/ablate.sh, pasted below from the same-box run)
The family times are per lane-forward (the two-lane split runs 64 + 64 images at bs 128).
Fill bytes per launch = tiles x k-tiles x (BM + BN) x 128 B (64 k of 16-bit A and W rows);
FLOP = 2 M N K. 'no-MFMA' time = fill + barriers + prologue/epilogue; 'no-fill' time = MFMA +
LDS fragment reads + epilogue.
"""
import math

NCU = 256
# model, role, M, N, K, (BM, BN), launches per forward, (full, no_fill, no_mfma) ms per forward
ROWS = [
    ("B/32 bs256", "qkv", 12800, 2304, 768, (240, 256), 12, (0.684, 0.464, 0.528)),
    ("B/32 bs256", "fc", 12800, 3072, 768, (160, 128), 11, (0.925, 0.515, 0.685)),
    ("B/32 bs256", "proj", 12800, 768, 3072, (160, 128), 11, (0.733, 0.413, 0.592)),
    ("B/32 bs256", "out", 12800, 768, 768, (160, 128), 11, (0.276, 0.182, 0.233)),
    ("L/14@336 bs128 (lane 64)", "qkv", 64 * 577, 3072, 1024, (256, 256), 24, (6.054, 3.537, 5.189)),
    ("L/14@336 bs128 (lane 64)", "fc", 64 * 577, 4096, 1024, (256, 256), 23, (7.732, 4.884, 6.743)),
    ("L/14@336 bs128 (lane 64)", "proj", 64 * 577, 1024, 4096, (256, 256), 23, (7.691, 4.521, 6.602)),
]


def main():
    print("| model | role | tiles | fill GB/fwd | no-MFMA ms | fill TB/s (GB/s/CU) | no-fill ms | MFMA-side PF/s | full PF/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for model, role, M, N, K, (bm, bn), L, (full, nofill, nomfma) in ROWS:
        tiles = math.ceil(M / bm) * (N // bn)
        fill = tiles * (K // 64) * (bm + bn) * 128 * L
        flop = 2.0 * M * N * K * L
        print(f"| {model} | {role} | {tiles} | {fill / 1e9:.2f} | {nomfma:.3f} | "
              f"{fill / nomfma / 1e9:.1f} ({fill / nomfma / 1e6 / NCU:.0f}) | {nofill:.3f} | "
              f"{flop / nofill / 1e12:.2f} | {flop / full / 1e12:.2f} |")


if __name__ == "__main__":
    main()
