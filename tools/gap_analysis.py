"""Idle time between kernels of the forward, from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- python bench.py ...
    python tools/gap_analysis.py gpurun_out/gaps

Takes the dispatches of the last N forwards (a forward starts at each im2col launch), and reports
per forward: span (first start -> last end), summed kernel time, and the idle gaps between
consecutive kernels (largest ones named), i.e. what a hipGraph / fewer launches could recover.
"""
import csv
import glob
import sys


def main(d, n_fwd=5):
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "im2col" in r[2]]
    if len(starts) < n_fwd + 1:
        n_fwd = len(starts) - 1
    for s, e in zip(starts[-n_fwd - 1:-1], starts[-n_fwd:]):
        seg = rows[s:e]
        # trailing head kernels belong to this forward; the next forward starts at im2col
        span = seg[-1][1] - seg[0][0]
        busy = sum(b - a for a, b, _ in seg)
        gaps = []
        for (a0, b0, n0), (a1, b1, n1) in zip(seg, seg[1:]):
            gaps.append((a1 - b0, n0[:50], n1[:50]))
        gaps.sort(reverse=True)
        pos = [g for g in gaps if g[0] > 0]
        print(f"kernels {len(seg)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us  "
              f"idle {(span-busy)/1e3:.1f} us  mean gap {sum(g[0] for g in pos)/max(1,len(pos))/1e3:.2f} us")
    for g in gaps[:8]:
        print(f"   {g[0]/1e3:7.2f} us  {g[1]} -> {g[2]}")


if __name__ == "__main__":
    main(sys.argv[1])
