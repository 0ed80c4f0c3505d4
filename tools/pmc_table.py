"""Table of the tools/pmc_gemm.sh counter passes (one row per GEMM case, averaged over its launches).

    python tools/pmc_table.py gpurun_out/pmc "qkv,out,fc,proj"

A case = one run of consecutive GEMM dispatches in dispatch order (tools/gemm_multi.py fills the
operands with other kernels between cases). Formulas (MI355X: 8 XCDs, 1024 SIMDs):
  clock       = GRBM_GUI_ACTIVE / 8 / duration
  MFMA busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)
  L2 hit      = TCC_HIT / (TCC_HIT + TCC_MISS)
  wait share  = SQ_WAIT_ANY / SQ_WAVE_CYCLES (wave-cycles spent waiting on any counter)
  LDS conflict= SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import csv
import sys
from collections import OrderedDict, defaultdict
from pathlib import Path


def load(d):
    disp = OrderedDict()
    for f in sorted(Path(d).glob("p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            key = (f.parent.name, int(r["Dispatch_Id"]))
            e = disp.setdefault(key, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                      "vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"],
                                      "lds": r["LDS_Block_Size"],
                                      "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9, "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def cases(disp):
    """per pass: the runs of consecutive GEMM dispatches, in dispatch order"""
    out, open_run = defaultdict(list), {}
    for (p, _), e in disp.items():
        if "gemm" in e["name"]:
            if not open_run.get(p):
                out[p].append([])
                open_run[p] = True
            out[p][-1].append(e)
        else:
            open_run[p] = False
    return out


def main():
    d, names = sys.argv[1], sys.argv[2].split(",")
    per = cases(load(d))
    rows = []
    for i, nm in enumerate(names):
        agg, meta = defaultdict(float), {}
        for p, runs in per.items():
            if i >= len(runs):
                continue
            for e in runs[i]:
                for k, v in e["c"].items():
                    agg[(p, k)] += v / len(runs[i])
                agg[(p, "dur")] += e["dur"] / len(runs[i])
                meta = {k: e[k] for k in ("name", "grid", "vgpr", "agpr", "lds")}

        def g(k):
            for (p, kk), v in agg.items():
                if kk == k:
                    return v
            return None

        def dur_of(k):
            for (p, kk), v in agg.items():
                if kk == k:
                    return agg.get((p, "dur"))
            return None

        gui, mfma, dur = g("GRBM_GUI_ACTIVE"), g("SQ_VALU_MFMA_BUSY_CYCLES"), dur_of("GRBM_GUI_ACTIVE")
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        wait, wcyc = g("SQ_WAIT_ANY"), g("SQ_WAVE_CYCLES")
        conf, ldsact = g("SQ_LDS_BANK_CONFLICT"), g("SQ_LDS_IDX_ACTIVE")
        rows.append((nm, meta, dur, gui / 8 / dur / 1e9 if gui and dur else None,
                     mfma / (1024 * gui / 8) if mfma and gui else None,
                     hit / (hit + miss) if hit is not None and miss else None,
                     wait / wcyc if wait and wcyc else None,
                     conf / ldsact if conf is not None and ldsact else None))
    print("| role | kernel template args (grid threads) | LDS B | us (under PMC) | clock GHz | MFMA busy | L2 hit | wait share | LDS conflict |")
    print("|---|---|---|---|---|---|---|---|---|")
    f = lambda v, fmt: (fmt % v) if v is not None else ""
    for nm, m, dur, clk, mf, l2, w, c in rows:
        kn = m.get("name", "")
        kn = kn[kn.find("<") + 1:kn.find(">")] if "<" in kn else kn
        print(f"| {nm} | {kn} ({m.get('grid', '')}) | {m.get('lds', '')} | "
              f"{f(dur * 1e6 if dur else None, '%.1f')} | {f(clk, '%.2f')} | {f(mf, '%.2f')} | {f(l2, '%.2f')} | "
              f"{f(w, '%.2f')} | {f(c, '%.3f')} |")


if __name__ == "__main__":
    main()
