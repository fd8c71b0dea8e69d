"""Per-kernel device time of a rocprofv3 kernel trace, grouped by kernel and grid: the mean
duration per distinct (kernel, grid) launch shape. Usage: kt_summary.py LABEL kernel_trace.csv"""
import collections
import csv
import sys

label, path = sys.argv[1], sys.argv[2]
d = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    key = (r["Kernel_Name"].split("(")[0].replace("thesia::", "")[:28], int(r["Grid_Size_X"]) // 256,
           int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    if "copyBuffer" in k[0] or "fillBuffer" in k[0]:
        continue
    print(label, k[0], k[1:], len(v), "%.1f us" % (sum(v) / len(v)))
