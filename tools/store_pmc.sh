#!/bin/bash
# L2-pollution check of the epilogue stores: FETCH_SIZE and WRITE_SIZE of the
# persistent c_fc tile (variant 62, M = 12,800) with the shipped library and with ab/nostore.so
# (CLIPVIT_ABLATE=3 build of gemm_pp.hip: no epilogue stores). Separate PMC pass per counter.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/store_pmc
cd /tmp && export TMPDIR=/tmp
for lib in shipped nostore; do
  L=""; [ $lib = nostore ] && L=$R/ab/nostore.so
  for c in FETCH_SIZE WRITE_SIZE; do
    CLIPVIT_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/store_pmc/${lib}_$c -o run -- \
      python3 $R/tools/gemm_ab.py "12800,3072,768,1" "62" 1 10 > $R/gpurun_out/store_pmc/${lib}_$c.txt 2>&1 \
      || { echo "pmc pass failed ($lib $c)"; tail -5 $R/gpurun_out/store_pmc/${lib}_$c.txt; exit 1; }
    grep "v62" $R/gpurun_out/store_pmc/${lib}_$c.txt
  done
done
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
for lib in ("shipped", "nostore"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = []
        for f in glob.glob(f"{R}/gpurun_out/store_pmc/{lib}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "gemm_ppp_kernel" in r.get("Kernel_Name", ""):
                    vals.append(float(r["Counter_Value"]))
        if vals:
            print(f"{lib:8s} {c:10s} dispatches {len(vals):3d} mean {sum(vals)/len(vals)/1e3:8.1f} MB (raw KB units / 1e3)")
PY
