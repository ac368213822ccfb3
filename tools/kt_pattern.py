"""Per-case fused-kernel launch durations (us) in launch order from tools/gpu_kt_repeat.sh output."""
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*")), key=lambda p: int(os.path.basename(p))):
    case = open(os.path.join(d, "case.txt")).read().strip()
    rows = []
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for name in ("k_admm3d", "k_dct8"):
        dur = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows if name in r["Kernel_Name"]]
        print(case, name, len(dur), dur[:24])
