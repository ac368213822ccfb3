"""Per-kernel duration summary of a rocprofv3 --kernel-trace run (real launches only).

Usage: python tools/prof_summary.py <dir with run_kernel_trace.csv> [out.md]

The rocprofv3 --stats table averages every launch, including the PCG launches that were
enqueued after convergence and returned at once (a device-side done flag) and the untimed
warm-up. This summary drops launches shorter than 5 % of the kernel's median, so its mean is
comparable with the per-launch HIP-event average bench.py reports for the timed region.
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main(d: str, out: str | None) -> None:
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    durs = defaultdict(list)
    full = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            full.setdefault(k, r["Kernel_Name"][:90])
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in durs.values())
    lines = ["| kernel | launches (all) | launches (real) | mean us (real) | median us | min us | max us | share |",
             "|---|---|---|---|---|---|---|---|"]
    for k, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        med = statistics.median(v)
        real = [x for x in v if x >= 0.05 * med]
        lines.append(f"| {k} | {len(v)} | {len(real)} | {statistics.mean(real):.1f} | {statistics.median(real):.1f} | "
                     f"{min(real):.1f} | {max(real):.1f} | {sum(v) / total:.3f} |")
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as fh:
            fh.write(f"rocprofv3 --kernel-trace summary of `{d}` (tools/prof_summary.py)\n\n" + txt + "\n\n")
            fh.write("\n".join(f"* {k}: `{n}`" for k, n in sorted(full.items())) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
