"""Mean per-dispatch PMC values from rocprofv3 counter_collection CSVs, grouped by kernel and grid.
Usage: pmc_summary.py counter_collection.csv [more.csv ...]"""
import collections
import csv
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("thesia::", "").replace("void ", "")[:40]
        key = (name, r.get("Grid_Size", ""))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in sorted(vals):
    c = vals[key]
    n = max(len(v) for v in c.values())
    parts = []
    for cn in sorted(c):
        m = sum(c[cn]) / len(c[cn])
        parts.append(f"{cn}={m:.4g}")
    wc = sum(c.get("SQ_WAVE_CYCLES", [0])) / max(len(c.get("SQ_WAVE_CYCLES", [1])), 1)
    extra = ""
    if wc:
        for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if cn in c:
                extra += f" {cn}/WC={sum(c[cn]) / len(c[cn]) / wc:.3f}"
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
            w = sum(c["SQ_WAVES"]) / len(c["SQ_WAVES"])
            extra += f" VALU/wave={sum(c['SQ_INSTS_VALU']) / len(c['SQ_INSTS_VALU']) / w:.1f}"
            extra += f" WC/wave={wc / w:.0f}"
    print(key[0], key[1], f"n={n}", " ".join(parts), extra)
