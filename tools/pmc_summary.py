"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes per kernel.

Usage: python tools/pmc_summary.py gpurun_out [profiles/<round>/pmc_traffic.json]

FETCH_SIZE / WRITE_SIZE are in KiB and come from the L2's memory-side request counters
(MI355X_MICROARCH.md §HBM). gfx950 under-reports wide streaming reads (FETCH_SIZE = 1/2 of the
bytes for 16-B lanes), and other widths are uncalibrated there, so the factors are measured here
with tools/pmc_calib.hip: known-size copies with 8-B and 16-B lanes. The mvtv kernels move
8-B lanes, so the 8-B factors are applied.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

NAMES = {"k_plane8": "dct_plane", "k_admm3d": "admm_fused", "k_admm3a": "admm_fused", "k_admm4a": "admm_fused4",
         "k_gather4a": "gather_Dt", "k_gather4b": "gather4_b", "k_edge3d": "edge_update", "k_gather3d": "gather_Dt", "k_dct8": "dct",
         "k_dct": "dct", "k_dctg": "dct", "k_tri": "dct_tri", "k_trig": "dct_tri", "k_trir": "dct_tri", "k_trigr": "dct_tri",
         "k_trisr": "dct_tris", "k_tris": "dct_tris",
         "k_cg3d": "pcg_fused3d", "k_edge_update": "edge_update", "k_gather": "gather_Dt",
         "k_apply_A": "pcg_apply_A", "k_pcg_update": "pcg_update", "k_pcg_pupdate": "pcg_direction",
         "k_pcg_init": "pcg_init", "copy8": "copy8", "copy16": "copy16"}


def short(kname: str) -> str:
    for k, v in NAMES.items():
        if re.search(r"\b" + k + r"\b", kname):
            if k == "k_cg3d":   # <WM, MODE, NWV>: 0 prologue, 1 first iteration, 2 (x untouched), 3 (x moved)
                mo = re.search(r"k_cg3d<\d+, (\d)", kname)
                mode = int(mo.group(1)) if mo else 2
                return {0: "pcg_init", 1: "pcg_fused3d_first", 2: "pcg_fused3d", 3: "pcg_fused3d_x"}[mode]
            if k in ("k_dct8", "k_dct") and re.search(r"k_dct8?<[^>]*true, true", kname):
                return "dct_first"   # the pass that forms b on load (FORMB)
            if k == "k_gather4b" and not re.search(r"k_gather4b<1, true>", kname):
                return "gather4_b_init"   # D^T u0 at a run's start (explicit u, no g_uprev: 3N), not the loop's 7N
            if k == "k_plane8" and re.search(r"k_plane8<\d+, 0, true>", kname):
                return "dct_plane_first"   # both in-plane forward passes, b formed on load
            return v
    return kname.split("(")[0]


def read_counter(d: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    # PCG launches enqueued after convergence return at once (done flag): drop them (< 2 % of the
    # kernel's largest launch) so the per-launch figure describes real iterations
    out, cnt = {}, {}
    for k, v in per.items():
        hi = max(v)
        real = [x for x in v if x >= 0.02 * hi] or v
        # the first pass forms b from oty, g_alpha, g_u (4N words: an ADMM run's first iteration, or after a rho
        # change) or from oty and the folded s (3N): one kernel, two traffic classes, split at the gap so each
        # launch class reconciles with its own model (mvtv_timing_get's dct_first / dct_first_fold)
        if k in ("dct_first", "dct_plane_first") and min(real) > 0 and max(real) / min(real) > 1.15:
            mid = 0.5 * (min(real) + max(real))
            lo, up = [x for x in real if x < mid], [x for x in real if x >= mid]
            out[k + "_fold"], cnt[k + "_fold"] = sum(lo) / len(lo), len(lo)
            out[k], cnt[k] = sum(up) / len(up), len(up)
            continue
        out[k] = sum(real) / len(real)
        cnt[k] = len(real)
    return out, cnt


def main(out_dir: str, dest: str | None):
    fetch, nf = read_counter(os.path.join(out_dir, "prof_fetch"), "FETCH_SIZE")
    write, nw = read_counter(os.path.join(out_dir, "prof_write"), "WRITE_SIZE")
    cf, _ = read_counter(os.path.join(out_dir, "calib_fetch"), "FETCH_SIZE")
    cw, _ = read_counter(os.path.join(out_dir, "calib_write"), "WRITE_SIZE")
    known = float(2 ** 28 * 8)   # bytes per launch of the calibration copies
    f8 = known / (cf["copy8"] * 1024) if cf.get("copy8") else None
    w8 = known / (cw["copy8"] * 1024) if cw.get("copy8") else None
    f16 = known / (cf["copy16"] * 1024) if cf.get("copy16") else None
    w16 = known / (cw["copy16"] * 1024) if cw.get("copy16") else None
    import datetime
    import subprocess
    try:
        head = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], text=True,
                                       cwd=os.path.dirname(os.path.abspath(__file__))).strip()
    except Exception:
        head = "?"
    out = {"_source": {"pass": f"rocprofv3 FETCH_SIZE + WRITE_SIZE passes of {out_dir} (tree {head})",
                       "date": datetime.date.today().isoformat()},
           "calibration": {"fetch_factor_8B": f8, "write_factor_8B": w8, "fetch_factor_16B": f16,
                           "write_factor_16B": w16},
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        base = k[:-5] if k.endswith("_fold") else k   # a split class's other counter may not have split (equal sizes)
        rd = fetch.get(k, fetch.get(base, 0.0)) * 1024 * (f8 or 1.0)
        wr = write.get(k, write.get(base, 0.0)) * 1024 * (w8 or 1.0)
        out["kernels"][k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
                             "launches_sampled": nf.get(k, 0)}
        out[k] = rd + wr
    txt = json.dumps(out, indent=1)
    print(txt)
    if dest:
        with open(dest, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
