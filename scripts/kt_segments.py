"""Display kernels per C5 group from a kernel trace of scripts/display_groups_ab.py (one stream):
the trace is cut at each group's spectrogram launch (stft*), then per segment every display
kernel's mean duration over its repeats. Usage: kt_segments.py kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
segs = []
for r in rows:
    name = r["Kernel_Name"].replace("void ", "").replace("thesia::", "").replace("(anonymous namespace)::", "")
    if "copyBuffer" in name or "fillBuffer" in name or "range_init" in name:
        continue
    cut = name.find(">(")
    name = name[:cut + 1] if cut >= 0 else name.split("(")[0]
    if name.startswith("stft"):
        segs.append(collections.OrderedDict())
        continue
    if not segs:
        continue
    segs[-1].setdefault(name[:52], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for i, s in enumerate(segs):
    tot = sum(sum(v) / len(v) for v in s.values())
    print("group %2d  sum %6.1f us : " % (i, tot) + "; ".join("%s %.1f" % (k, sum(v) / len(v)) for k, v in s.items()))
