"""Print the per-kernel stats of a rocprofv3 --kernel-trace --stats directory (tools/kt_only.sh)."""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
f = next(d.rglob("*kernel_stats.csv"))
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f'{r["Name"][:96]:96s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:8.1f}us {100 * float(r["TotalDurationNs"]) / tot:5.1f}%')
