"""Per-launch device times of a rocprofv3 kernel trace in launch order, one line per distinct
(kernel, grid) shape in order of first appearance: mean duration, count. For runs that process
display groups one after another (scripts/display_groups_ab.py with THESIA_RENDER_STREAMS=1).
Usage: kt_groups.py kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = collections.OrderedDict()
for r in rows:
    name = r["Kernel_Name"]
    if "copyBuffer" in name or "fillBuffer" in name:
        continue
    name = name.replace("void ", "").replace("thesia::", "")
    cut = name.find(">(")
    name = name[:cut + 1] if cut >= 0 else re.sub(r"\(.*$", "", name)
    key = (name[:60], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]),
           int(r["Grid_Size_Z"]), int(r["Workgroup_Size_X"]))
    d.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print("%-60s blocks %5d x %4d x %4d wg %4d  n %3d  mean %7.1f us  min %7.1f" % (k + (len(v), sum(v) / len(v), min(v))))
