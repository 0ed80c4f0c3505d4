"""Host-only: per-role medians of the PMC passes of `tools/r06_runs.sh phases` (default bench,
one counter set per rocprofv3 run), as a markdown table, with derived per-CU rates.

    python tools/r06_pmc_phases.py gpurun_out/r06_phases > profiles/r06/pmc_roles.md

Roles come from the dispatch order of the forward (tools/summarize_profiles.py roles_by_queue).
SQ_* counters are summed over the chip (SQ_WAVE_CYCLES, SQ_WAIT_* and SQ_ACTIVE_* in quad-cycles,
per MI355X_MICROARCH.md), TA/TCP *_sum over the 256 TA / TCP instances, *_avr averaged.
"""
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from summarize_profiles import roles_by_queue  # noqa: E402

ROLES = ["qkv", "out", "fc", "proj", "patch_gemm", "attention", "ln1", "ln2"]


def load(d: Path):
    trace = list(csv.DictReader(open(d / "run_kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    roles = roles_by_queue(trace)
    role_of = {r["Dispatch_Id"]: role for r, role in zip(trace, roles)}
    dur = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in trace}
    vals = defaultdict(lambda: defaultdict(list))
    seen = defaultdict(dict)
    for r in csv.DictReader(open(d / "run_counter_collection.csv")):
        seen[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    for disp, cs in seen.items():
        role = role_of.get(disp)
        if role in ROLES:
            for k, v in cs.items():
                vals[role][k].append(v)
            vals[role]["_us"].append(dur.get(disp, 0.0))
    return vals


def main():
    src = Path(sys.argv[1])
    med = defaultdict(dict)
    for p in sorted(src.glob("pmc*")):
        if not p.is_dir():
            continue
        for role, cs in load(p).items():
            for k, v in cs.items():
                med[role][k] = statistics.median(v) if k != "_us" else statistics.median(v)
    counters = sorted({k for r in med.values() for k in r if k != "_us"})
    print("| counter (median per dispatch) | " + " | ".join(r for r in ROLES if r in med) + " |")
    print("|---|" + "---|" * sum(1 for r in ROLES if r in med))
    for c in counters:
        print(f"| {c} | " + " | ".join(f"{med[r].get(c, float('nan')):.4g}" for r in ROLES if r in med) + " |")
    # derived: per-CU view over the dispatch's GPU-active cycles (GRBM_GUI_ACTIVE / 8 XCDs)
    print()
    print("| derived | " + " | ".join(r for r in ROLES if r in med) + " |")
    print("|---|" + "---|" * sum(1 for r in ROLES if r in med))

    def row(name, fn):
        out = []
        for r in ROLES:
            if r not in med:
                continue
            try:
                out.append(f"{fn(med[r]):.3g}")
            except (KeyError, ZeroDivisionError, ValueError):
                out.append("n/a")
        print(f"| {name} | " + " | ".join(out) + " |")

    cyc = lambda m: m["GRBM_GUI_ACTIVE"] / 8.0  # noqa: E731 (per-XCD active cycles of the dispatch)
    row("active cycles (GRBM_GUI_ACTIVE / 8)", cyc)
    row("TA busy share (TA_TA_BUSY_sum / 256 TAs / cycles)", lambda m: m["TA_TA_BUSY_sum"] / 256 / cyc(m))
    row("TCP pending-data stall share (TCP_PENDING_STALL_CYCLES_sum / 256 / cycles)",
        lambda m: m["TCP_PENDING_STALL_CYCLES_sum"] / 256 / cyc(m))
    row("TCP stalled by TCR share (TCP_TCR_TCP_STALL_CYCLES_sum / 256 / cycles)",
        lambda m: m["TCP_TCR_TCP_STALL_CYCLES_sum"] / 256 / cyc(m))
    row("mean L2 read latency, cycles (READ_REQ_LATENCY / READ_REQ)",
        lambda m: m["TCP_TCC_READ_REQ_LATENCY_sum"] / m["TCP_TCC_READ_REQ_sum"])
    row("L2 read requests in flight per CU (Little)",
        lambda m: m["TCP_TCC_READ_REQ_LATENCY_sum"] / 256 / cyc(m))
    row("MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / cycles)",
        lambda m: m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc(m))
    row("LDS-issue-stall share of wave cycles (SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES)",
        lambda m: m["SQ_WAIT_INST_LDS"] / m["SQ_WAVE_CYCLES"])
    row("waiting (s_waitcnt / barrier) share (SQ_WAIT_ANY / SQ_WAVE_CYCLES)", lambda m: m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"])
    row("issue-stall share (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)", lambda m: m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"])
    row("LDS instructions per VMEM instruction", lambda m: m["SQ_INSTS_LDS"] / m["SQ_INSTS_VMEM"])


if __name__ == "__main__":
    main()
