"""Average SQ/TCC counter values per kernel from tools/gpu_counters.sh output (real launches only).

Usage: python tools/ctr_summary.py <dir> [--full]
--full keys the table by the kernel's full template instantiation (one row per k_dct8<...> variant) instead of the
bench's timing buckets, and adds the wave-cycle shares: SQ_WAIT_INST_ANY (issue stalls), SQ_WAIT_ANY (waits on
memory / counters), SQ_ACTIVE_INST_ANY, as fractions of SQ_WAVE_CYCLES."""
import csv
import glob
import sys
from collections import defaultdict

sys.path.insert(0, "tools")
from pmc_summary import short  # noqa: E402

full = "--full" in sys.argv
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/ctr*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "") if full else short(row["Kernel_Name"])
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    d = vals[k]
    ref = d.get("SQ_WAVES") or d.get("GRBM_GUI_ACTIVE") or next(iter(d.values()))
    hi = max(ref)
    keep = [i for i, v in enumerate(ref) if v >= 0.5 * hi]
    print(k)
    mean = {}
    for c in sorted(d):
        v = d[c]
        sel = [v[i] for i in keep if i < len(v)] or v
        mean[c] = sum(sel) / len(sel)
        print(f"   {c:28s} {mean[c]:16.1f}   (n={len(sel)})")
    wc = mean.get("SQ_WAVE_CYCLES")
    if full and wc:
        shares = {c: mean[c] / wc for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY") if c in mean}
        print("   shares of wave cycles: " + ", ".join(f"{c[3:]} {s:.2f}" for c, s in shares.items()))
    if full and mean.get("SQ_INSTS_VALU"):
        print(f"   SALU:VALU {mean.get('SQ_INSTS_SALU', 0.0) / mean['SQ_INSTS_VALU']:.2f}")
