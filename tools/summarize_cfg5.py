"""Config-5 (MX-fp8, bs 512, two lanes of 256) rocprofv3 passes -> profiles/<tag>_cfg5_summary.md.

    python tools/summarize_cfg5.py gpurun_out/cfg5prof r04

Roles come from summarize_profiles.roles_by_queue (per hardware queue, dispatch order); each GEMM
role is split by operand format: "mx" for the MX-fp8 kernels (gemm_mx8*), "16" for the bf16
blocks the default keeps (0, 1, 10, 11 MLP; 1, 11 attention roles). FLOP rates are against the
role's own dense peak (5.0332 PF/s MX-fp8, 2.5166 PF/s bf16). MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs x GRBM_GUI_ACTIVE / 8), wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES, L2 hit = TCC_HIT / (HIT +
MISS), each from its own rocprofv3 pass of the same command. Dispatches of the timed loop run two
lanes concurrently ("concurrent"); bench.py's profile pass runs one lane alone ("isolated").
"""
import shutil
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from summarize_profiles import ROOT, fc_split_rows, isolated_flags, load_rows, roles_by_queue  # noqa: E402

D, LANE = 768, 256
M = LANE * 50
SHAPES = {"qkv": (M, 3 * D, D), "out": (M, D, D), "fc": (M, 4 * D, D), "proj": (M, D, 4 * D)}


def key_of(role, name):
    if role in ("qkv", "out", "fc", "fc_tail", "proj"):
        return f"{role} {'mx' if 'mx8' in name else '16'}"
    return role


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    prof = ROOT / "profiles"
    shutil.copyfile(next((src / "kt").rglob("*kernel_stats.csv")), prof / f"{tag}_cfg5_kernel_stats.csv")
    trace = load_rows(next((src / "kt").rglob("*kernel_trace.csv")))
    roles = roles_by_queue(trace)
    iso = isolated_flags(trace)
    dur, dur_c = defaultdict(list), defaultdict(list)
    for r, role, solo in zip(trace, roles, iso):
        (dur if solo else dur_c)[key_of(role, r["Kernel_Name"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

    def pmc(kind, counter):
        d = src / kind
        if not d.exists():
            return {}
        rows = [r for r in load_rows(next(d.rglob("*counter_collection.csv"))) if r.get("Counter_Name") == counter]
        acc = defaultdict(list)
        for r, role in zip(rows, roles_by_queue(rows, key="Dispatch_Id")):
            acc[key_of(role, r["Kernel_Name"])].append(float(r["Counter_Value"]))
        return acc

    busy, gui = pmc("mfma", "SQ_VALU_MFMA_BUSY_CYCLES"), pmc("mfma", "GRBM_GUI_ACTIVE")
    wcyc, wait = pmc("mfma", "SQ_WAVE_CYCLES"), pmc("mfma", "SQ_WAIT_ANY")
    hit, miss = pmc("l2", "TCC_HIT_sum"), pmc("l2", "TCC_MISS_sum")

    def mean(v):
        return sum(v) / len(v) if v else float("nan")
    m1 = fc_split_rows(M)
    lines = [f"# {tag}: rocprofv3 summary of `python bench.py --dtype mxfp8 --batch 512` (BASELINE config 5; two lanes of 256 images)", "",
             "Per role and operand format (mx = MX-fp8 scaled MFMA, 16 = the bf16 blocks the default keeps). avg us:",
             "isolated dispatches (bench.py's one-lane profile pass) where present, else the concurrent ones (both",
             "lanes on the GPU, the timed loop). frac = the launch's FLOPs / avg / the format's dense peak (5.0332 PF/s",
             "MX-fp8, 2.5166 PF/s bf16). MFMA busy, wait and L2 hit: one rocprofv3 --pmc pass each (see",
             "tools/summarize_cfg5.py).", "",
             "| role | isolated dispatches | avg us | concurrent dispatches | concurrent avg us | TFLOP/s | frac of peak | MFMA busy | wait | L2 hit |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for k in sorted(set(dur) | set(dur_c), key=lambda k: -sum(dur.get(k, [])) - sum(dur_c.get(k, []))):
        d, dc = dur.get(k, []), dur_c.get(k, [])
        avg = mean(d) if d else mean(dc)
        role, fmt = (k.split(" ") + [""])[:2]
        tf = fr = ""
        if role in SHAPES or role == "fc_tail":
            m, n, kk = SHAPES.get(role, SHAPES["fc"])
            if fmt == "16" and role == "fc" and m1:
                m = m1
            if role == "fc_tail":
                m = M - m1
            fl = 2 * m * n * kk
            peak = 5.0332e15 if fmt == "mx" else 2.5166e15
            tf, fr = f"{fl / (avg * 1e-6) / 1e12:.0f}", f"{fl / (avg * 1e-6) / peak:.3f}"
        mb = mean(busy.get(k, [])) / (1024 * mean(gui.get(k, [])) / 8) if busy.get(k) else float("nan")
        wt = mean(wait.get(k, [])) / mean(wcyc.get(k, [])) if wait.get(k) else float("nan")
        h, ms = mean(hit.get(k, [])), mean(miss.get(k, []))
        l2 = h / (h + ms) if hit.get(k) else float("nan")
        lines.append(f"| {k} | {len(d)} | {avg:.1f} | {len(dc)} | {mean(dc) if dc else float('nan'):.1f} | {tf} | {fr} "
                     f"| {mb:.3f} | {wt:.3f} | {l2:.3f} |")
    (prof / f"{tag}_cfg5_summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
