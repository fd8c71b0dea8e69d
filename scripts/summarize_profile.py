"""Copy a rocprofv3 run (scripts/profile.sh output under gpurun_out/) into profiles/<tag>/ and
derive the per-launch HBM traffic of the STFT kernel from the PMC passes.

FETCH_SIZE / WRITE_SIZE are in KiB summed over the launch. On gfx950 FETCH_SIZE reports half
the bytes of a 16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is exact for wide streaming stores. Usage:
    python scripts/summarize_profile.py <tag> <workload_key> [gpurun_out dir]
"""
from __future__ import annotations

import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, match="stft"):
    vals = collections.defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "VGPR_Count",
                                      "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size")}
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}, meta


def main():
    tag, wkey = sys.argv[1], sys.argv[2]
    src = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    summary = {"workload_key": wkey}
    kt = os.path.join(src, "prof_kt", "kt_kernel_stats.csv")
    if os.path.exists(kt):
        shutil.copy(kt, os.path.join(dst, "kernel_stats.csv"))
        rows = list(csv.DictReader(open(kt)))
        summary["kernel_stats"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs")}
                                   for r in rows]
    counters = {}
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d, "pmc_counter_collection.csv")
        if d.startswith("prof_pmc") and os.path.exists(p):
            avg, n, meta = per_kernel(p)
            counters.update(avg)
            summary["dispatch_meta"] = meta
            shutil.copy(p, os.path.join(dst, d.replace("prof_", "") + ".csv"))
    summary["pmc_avg_per_launch"] = counters
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        fetch = counters["FETCH_SIZE"] * 1024 * 2  # KiB, gfx950 half-count correction
        write = counters["WRITE_SIZE"] * 1024
        summary["hbm_bytes_per_launch"] = fetch + write
        summary["fetch_bytes_corrected"] = fetch
        summary["write_bytes"] = write
        tj = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        try:
            allt = json.load(open(tj))
        except (OSError, ValueError):
            allt = {}
        allt[wkey] = {"hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch,
                      "write_bytes": write, "profile": tag}
        json.dump(allt, open(tj, "w"), indent=1)
    for name in ("bench.log", "prof_kt.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            lines = [ln for ln in open(p) if ln.startswith("{")]
            if lines:
                summary.setdefault("bench_lines", {})[name] = json.loads(lines[-1])
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps({k: summary[k] for k in summary if k not in ("bench_lines",)}, indent=1))


if __name__ == "__main__":
    main()
