"""Host-only: per-kernel median PMC values from the rocprofv3 .db files of tools/r05_runs.sh pmc
(gpurun_out/r05_pmc/k<kind>/p<pass>/) -> a markdown table on stdout."""
import collections
import glob
import sqlite3
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05_pmc"
KIND = {"0": "v72 row-major A, W", "1": "v72 blocked A + W", "2": "v62 copy", "cproj": "c_proj v82"}
rows = {}
for kind in KIND:
    vals = collections.defaultdict(list)
    for db in sorted(glob.glob(f"{root}/k{kind}/p*/**/*.db", recursive=True)):
        con = sqlite3.connect(db)
        q = "select kernel_name, counter_name, value, dispatch_id from counters_collection"
        per = collections.defaultdict(float)
        for name, cnt, v, d in con.execute(q):
            if "gemm" not in name and "ppp" not in name:
                continue
            per[(cnt, d)] += v
        for (cnt, d), v in per.items():
            vals[cnt].append(v)
    rows[kind] = {k: statistics.median(v) for k, v in vals.items()}
cnts = sorted({c for r in rows.values() for c in r})
print("| counter (median per dispatch) | " + " | ".join(KIND[k] for k in KIND) + " |")
print("|---|" + "---|" * len(KIND))
for c in cnts:
    print(f"| {c} | " + " | ".join(f"{rows[k].get(c, float('nan')):.4g}" for k in KIND) + " |")
