"""Per-case mean FETCH_SIZE (bytes, gfx950 factor 2 for 8-B lanes) of the main kernels from
tools/gpu_ab_fetch.sh output: python tools/ab_summary.py gpurun_out/ab"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p)) if os.path.basename(p).isdigit() else 0):
    if not os.path.isdir(d):
        continue
    case = open(os.path.join(d, "case.txt")).read().strip() if os.path.exists(os.path.join(d, "case.txt")) else d
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "fetch", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == "FETCH_SIZE":
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024 * 2)
    out = {k: round(statistics.median(v) / 1e9, 3) for k, v in vals.items() if k in ("admm_fused", "dct", "dct_first", "gather_Dt", "edge_update")}
    print(case, "FETCH GB (median per launch):", out)
