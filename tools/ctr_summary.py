"""Average SQ/TCC counter values per kernel from tools/gpu_counters.sh output (real launches only)."""
import csv
import glob
import sys
from collections import defaultdict

sys.path.insert(0, "tools")
from pmc_summary import short  # noqa: E402

vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/ctr*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    d = vals[k]
    ref = d.get("SQ_WAVES") or d.get("GRBM_GUI_ACTIVE") or next(iter(d.values()))
    hi = max(ref)
    keep = [i for i, v in enumerate(ref) if v >= 0.5 * hi]
    print(k)
    for c in sorted(d):
        v = d[c]
        sel = [v[i] for i in keep if i < len(v)] or v
        print(f"   {c:28s} {sum(sel) / len(sel):16.1f}   (n={len(sel)})")
