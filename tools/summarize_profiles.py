"""Turn a tools/profile_round.sh output directory into committed summaries under profiles/.

    python tools/summarize_profiles.py gpurun_out/prof r02 [images_per_launch] [--summary-only]
writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim), profiles/<tag>_summary.md
(per-kernel-role averages, MFMA TFLOP/s, PMC bytes per launch) and updates
profiles/pmc_traffic.json (read by bench.py's roofline.traffic).

Kernel roles are assigned from the dispatch order of one forward (per layer: qkv GEMM,
attention, out GEMM, layernorm, fc GEMM, proj GEMM, layernorm), which is how out- and
proj-GEMM dispatches of the same template instance are told apart. The order is followed per
hardware queue: a batch split over the two lane streams interleaves two forwards in time.
A dispatch is "isolated" when no dispatch of another queue overlaps it (bench.py's
clipvit_profile_forward pass: one lane, serialised — what the bench's roofline times) and
"concurrent" otherwise (the timed loop's two lanes share the GPU).

images_per_launch: images per GEMM launch (bs 256 with the default two-lane split: 128).
--summary-only: write profiles/<tag>_summary.md only (A/B arms: no kernel_stats copy, no
fc_traffic / pmc_traffic JSON).
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def gemm_like(name):
    return "gemm" in name


def roles_for_trace(rows):
    """Assign a role to every dispatch of the encoder forward, by order. Between two attention
    dispatches a block runs out_proj, [ln_2], c_fc (one launch, or main + tail with the
    whole-round row split), c_proj, [ln_1] (the LayerNorm passes exist only on the unfolded
    path) and the next block's QKV."""
    out = []
    seg = None  # GEMMs seen since the last attention
    for r in rows:
        n = r["Kernel_Name"]
        if "cast_pixels" in n:
            out.append("pixel_cast"); continue
        if gemm_like(n) and "EPI_PATCH" not in n and n.rstrip(")").split(">")[0].split(",")[-1].strip() in ("14", "16", "32"):
            out.append("patch_gemm"); seg = None; continue
        if "im2col" in n:
            out.append("im2col"); continue
        if out and out[-1] == "im2col" and gemm_like(n):  # the explicit patch GEMM on the im2col matrix
            out.append("patch_gemm"); seg = None; continue
        if "embed_ln" in n or "embed_stats" in n:
            out.append("embed"); seg = [] ; continue
        if "gather_cls" in n:  # last block on class-token rows (cls_tail)
            out.append("cls_tail"); seg = "tail"; continue
        if seg == "tail" and (gemm_like(n) or "layernorm" in n):
            out.append("cls_tail"); continue
        if "cls_ln_proj" in n:
            out.append("head_proj"); seg = None; continue
        if "logits_kernel" in n:
            out.append("head_logits"); continue
        if "seg_softmax" in n:
            out.append("head_softmax"); continue
        if "attention" in n:
            out.append("attention"); seg = []; continue
        if isinstance(seg, list) and "layernorm" in n:
            out.append("ln2" if len(seg) == 1 else "ln1"); continue
        if isinstance(seg, list) and gemm_like(n):
            seg.append(n)
            out.append(None)  # resolved below
            continue
        out.append("other")
    # resolve the GEMMs of each segment: [qkv] after embed; out, fc, [fc_tail], proj, qkv after attention
    res, i = list(out), 0
    cur = []
    def flush(idx_list, after_attention):
        names = (["out", "fc", "proj", "qkv"] if len(idx_list) == 4 else ["out", "fc", "fc_tail", "proj", "qkv"]) \
            if after_attention else ["qkv"]
        for k, ix in enumerate(idx_list):
            res[ix] = names[k] if k < len(names) else "other"
    after_att = False
    for ix, (r, role) in enumerate(zip(rows, out)):
        if role == "attention" or role == "cls_tail" or role == "head_proj":
            flush(cur, after_att); cur = []; after_att = role == "attention"
        elif role == "embed":
            flush(cur, after_att); cur = []; after_att = False
        elif role is None:
            cur.append(ix)
    flush(cur, after_att)
    return [x if x is not None else "other" for x in res]


def load_rows(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r.get("Start_Timestamp") or r.get("Dispatch_Id") or 0))
    return rows


def roles_by_queue(rows, key="Start_Timestamp"):
    """roles_for_trace applied to each hardware queue's dispatches in order."""
    roles = [None] * len(rows)
    byq = defaultdict(list)
    for i, r in enumerate(rows):
        byq[r.get("Queue_Id", "0")].append(i)
    for idx in byq.values():
        idx.sort(key=lambda i: int(rows[i][key]))
        for i, role in zip(idx, roles_for_trace([rows[i] for i in idx])):
            roles[i] = role
    return roles


def isolated_flags(rows):
    """True for a dispatch that no dispatch of another queue overlaps in time."""
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "0"), i)
                 for i, r in enumerate(rows)))
    iso = [True] * len(rows)
    active = []  # (end, queue, index) of dispatches still running
    for s0, e0, q, i in ev:
        active = [a for a in active if a[0] > s0]
        for e1, q1, j in active:
            if q1 != q:
                iso[i] = iso[j] = False
        active.append((e0, q, i))
    return iso


def fc_split_rows(M, N=3072, ncu=256):
    """Main-launch rows of clipvit.hip gemm()'s whole-round row split (0 = no split)."""
    nN = N // 256
    t256 = (M + 255) // 256 * nN
    R, rem = divmod(t256, ncu)
    m1 = R * ncu // nN * 256
    return m1 if R >= 1 and 0 < rem and 2 * rem <= ncu and 0 < m1 < M else 0


def main():
    only = "--summary-only" in sys.argv
    argv = [x for x in sys.argv if x != "--summary-only"]
    src, tag = Path(argv[1]), argv[2]
    lane_b = int(argv[3]) if len(argv) > 3 else 128
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    kt = next((src / "kt").rglob("*kernel_stats.csv"))
    if not only:
        shutil.copyfile(kt, prof / f"{tag}_kernel_stats.csv")
    trace = load_rows(next((src / "kt").rglob("*kernel_trace.csv")))
    roles = roles_by_queue(trace)
    iso = isolated_flags(trace)
    dur, dur_c = defaultdict(list), defaultdict(list)
    for r, role, solo in zip(trace, roles, iso):
        (dur if solo else dur_c)[role].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

    def pmc(kind, counter=None):
        """per role: the counter's value per dispatch (rows of other counters of a multi-counter
        pass are dropped before the roles are assigned, so every dispatch appears once)"""
        d = src / kind
        if not d.exists():
            return {}
        f = next(d.rglob("*counter_collection.csv"))
        rows = [r for r in load_rows(f) if counter is None or r.get("Counter_Name") == counter]
        rr = roles_by_queue(rows, key="Dispatch_Id")
        acc = defaultdict(list)
        for r, role in zip(rows, rr):
            acc[role].append(float(r["Counter_Value"]))
        return acc

    fetch, write = pmc("fetch"), pmc("write")
    busy, gui = pmc("mfma", "SQ_VALU_MFMA_BUSY_CYCLES"), pmc("mfma", "GRBM_GUI_ACTIVE")
    wcyc, wait = pmc("mfma", "SQ_WAVE_CYCLES"), pmc("mfma", "SQ_WAIT_ANY")
    hit, miss = pmc("l2", "TCC_HIT_sum"), pmc("l2", "TCC_MISS_sum")

    def mean(v):
        return sum(v) / len(v) if v else float("nan")
    M, D = lane_b * 50, 768
    # (rows, N, K) of each GEMM role per launch; c_fc with the whole-round row split: the main
    # launch covers rows [0, m1), the tail launch the rest
    shapes = {"qkv": (M, 3 * D, D), "out": (M, D, D), "proj": (M, D, 4 * D), "patch_gemm": (lane_b * 49, D, 3072)}
    # the round split is off by default since c_fc runs on the 160x128 tile: only when the trace
    # holds c_fc tail launches does the main launch cover fewer rows
    m1 = fc_split_rows(M) if "fc_tail" in roles else 0
    shapes["fc"] = (m1, 4 * D, D) if m1 else (M, 4 * D, D)
    if m1:
        shapes["fc_tail"] = (M - m1, 4 * D, D)
    flops = {r: 2 * m * n * k for r, (m, n, k) in shapes.items()}
    # algorithmic bytes per launch: A once, W once, 16-bit C once
    algo = {r: 2 * (m * k + n * k + m * n) for r, (m, n, k) in shapes.items()}
    lines = [f"# {tag}: rocprofv3 summary of `python bench.py` (ViT-B/32, bs 256, fp16 MFMA operands, fp32 pixels; {lane_b} images per launch)", "",
             "avg us / TFLOP/s: isolated dispatches (bench.py's serialised profile pass, what its roofline",
             "times); concurrent us: the timed loop's dispatches, two lanes sharing the GPU. TFLOP/s = the",
             "launch's own FLOPs / isolated average. Algorithmic MB = A + W + C (16-bit) once. PMC MB =",
             "2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction; L2 misses served from the Infinity Cache are",
             "counted, writes still dirty in L2 at kernel end are not). Counter passes (one rocprofv3 run",
             "each, same command): MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8",
             "XCDs); MFMA busy x 2.5166 PF/s = the MFMA-issue rate the counters saw; wait = SQ_WAIT_ANY /",
             "SQ_WAVE_CYCLES (wave-cycles parked on a counter or barrier); L2 hit = TCC_HIT / (HIT + MISS).", "",
             "PMC GB/s = (FETCH_SIZE x2 + WRITE_SIZE) / avg: the bytes the L2 exchanged with the fabric",
             "(HBM or Infinity Cache) per second, against the 8 TB/s HBM3E peak (≈6.3 TB/s achievable).", "",
             "| role | isolated dispatches | avg us | TFLOP/s | frac of 2.5166 PF | concurrent avg us | FETCH_SIZE x2 (MB) | WRITE_SIZE (MB) | PMC GB/s | frac of 8 TB/s | algorithmic MB | PMC / algorithmic | MFMA busy | wait | L2 hit |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for role in sorted(set(dur) | set(dur_c), key=lambda k: -sum(dur.get(k, [])) - sum(dur_c.get(k, []))):
        d = dur.get(role) or dur_c[role]
        avg = sum(d) / len(d)
        dc = dur_c.get(role, [])
        cavg = f"{sum(dc) / len(dc):.1f}" if dc else ""
        tf = f"{flops[role] / (avg * 1e-6) / 1e12:.0f}" if role in flops else ""
        fr = f"{flops[role] / (avg * 1e-6) / 2.5166e15:.3f}" if role in flops else ""
        mb = mean(busy.get(role, [])) / (1024 * mean(gui.get(role, [])) / 8) if busy.get(role) else float("nan")
        wt = mean(wait.get(role, [])) / mean(wcyc.get(role, [])) if wait.get(role) else float("nan")
        h, m_ = mean(hit.get(role, [])), mean(miss.get(role, []))
        l2 = h / (h + m_) if hit.get(role) else float("nan")
        fb = 2 * sum(fetch[role]) / len(fetch[role]) * 1024 / 1e6 if fetch.get(role) else float("nan")
        wb = sum(write[role]) / len(write[role]) * 1024 / 1e6 if write.get(role) else float("nan")
        traffic[role] = {"avg_us": avg, "read_bytes": fb * 1e6, "write_bytes": wb * 1e6, "mfma_busy": mb,
                         "wait_share": wt, "l2_hit": l2}
        al = f"{algo[role] / 1e6:.1f}" if role in algo else ""
        ratio = f"{(fb + wb) * 1e6 / algo[role]:.2f}" if role in algo else ""
        gbs = (fb + wb) * 1e6 / (avg * 1e-6) / 1e9
        lines.append(f"| {role} | {len(dur.get(role, []))} | {avg:.1f} | {tf} | {fr} | {cavg} | {fb:.1f} | {wb:.1f} | {gbs:.0f} | {gbs / 8000:.2f} | {al} | {ratio} "
                     f"| {mb:.3f} | {wt:.3f} | {l2:.3f} |")
    if "fc_tail" in traffic:  # one c_fc invocation = main + tail launch
        a, b = traffic["fc"], traffic.pop("fc_tail")
        wa, wb_ = a["avg_us"], b["avg_us"]  # time-weighted counter shares
        traffic["fc"] = {k: a[k] + b[k] for k in ("avg_us", "read_bytes", "write_bytes")}
        for k in ("mfma_busy", "wait_share", "l2_hit"):
            traffic["fc"][k] = (a[k] * wa + b[k] * wb_) / (wa + wb_)
        t = traffic["fc"]
        fl, al = flops["fc"] + flops["fc_tail"], algo["fc"] + algo["fc_tail"]
        gbs = (t['read_bytes'] + t['write_bytes']) / (t['avg_us'] * 1e-6) / 1e9
        lines.append(f"| fc (main + tail) | | {t['avg_us']:.1f} | {fl / (t['avg_us'] * 1e-6) / 1e12:.0f} | "
                     f"{fl / (t['avg_us'] * 1e-6) / 2.5166e15:.3f} | | "
                     f"{t['read_bytes'] / 1e6:.1f} | {t['write_bytes'] / 1e6:.1f} | {gbs:.0f} | {gbs / 8000:.2f} | {al / 1e6:.1f} | "
                     f"{(t['read_bytes'] + t['write_bytes']) / al:.2f} | {t['mfma_busy']:.3f} | {t['wait_share']:.3f} | "
                     f"{t['l2_hit']:.3f} |")
    (prof / f"{tag}_summary.md").write_text("\n".join(lines) + "\n")
    if only:
        return
    mlp = [traffic[r] for r in ("fc", "proj") if r in traffic]
    entry = {"mlp_gemm_bytes_per_launch": sum(t["read_bytes"] + t["write_bytes"] for t in mlp) / len(mlp),
             "mlp_gemm_avg_us": sum(t["avg_us"] for t in mlp) / len(mlp), "source": f"profiles/{tag}_summary.md",
             "note": "HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE reports half of wide streaming reads); Infinity-Cache hits are included by the counters"}
    if "fc" in traffic:  # bench.py --traffic-json: the dominant kernel's own PMC bytes per launch
        t = traffic["fc"]
        fl = flops["fc"] + flops.get("fc_tail", 0)
        (prof / f"{tag}_fc_traffic.json").write_text(json.dumps({
            "fc_gemm_bytes_per_launch": t["read_bytes"] + t["write_bytes"], "fc_gemm_avg_us": t["avg_us"],
            "fc_gemm_algorithmic_bytes": algo["fc"] + algo.get("fc_tail", 0),
            "fc_gemm_frac_rocprof": fl / (t["avg_us"] * 1e-6) / 2.5166e15,
            "fc_gemm_mfma_busy": t["mfma_busy"], "fc_gemm_wait_share": t["wait_share"], "fc_gemm_l2_hit": t["l2_hit"],
            "source": f"profiles/{tag}_summary.md (rocprofv3 kernel trace + --pmc FETCH_SIZE / WRITE_SIZE / MFMA-busy / L2 passes of bench.py)"}, indent=1))
    pj = prof / "pmc_traffic.json"
    data = json.loads(pj.read_text()) if pj.exists() else {}
    entry["images_per_launch"] = lane_b
    data["ViT-B/32|256"] = entry
    pj.write_text(json.dumps(data, indent=1))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
