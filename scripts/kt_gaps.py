"""Gaps between a C5 step's last spectrogram launch and its first display launch (kernel trace of
bench.py --workload c5): the host's range readback + exchange + display planning between the
phases. Usage: kt_gaps.py kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gaps, in_disp, lse = [], False, None
for r in rows:
    n = r["Kernel_Name"]
    if "stft" in n:
        in_disp, lse = False, int(r["End_Timestamp"])
    elif ("grey_vert" in n or "resize_h" in n or "render_stripe" in n) and not in_disp and lse is not None:
        gaps.append((int(r["Start_Timestamp"]) - lse) / 1e3)
        in_disp = True
print("spectrogram -> display gaps (us):", [round(g, 1) for g in gaps])
