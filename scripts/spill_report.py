"""Where a kernel's scratch spill instructions sit: for each stft3/stft5 instantiation in a
device assembly file (hipcc --cuda-device-only -S), the scratch loads / stores in total and
inside each loop (a block range closed by a backward branch). Diagnosis aid."""
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "Li1024E"
for m in re.finditer(r"\n(_ZN6thesia\d+stft\w*_kernel\w*):[^\n]*\n(.*?)\.Lfunc_end", src, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    lines = body.split("\n")
    labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\w+:", l)}
    loops = []
    for i, l in enumerate(lines):
        b = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if b and b.group(1) in labels and labels[b.group(1)] < i:
            loops.append((labels[b.group(1)], i))
    tot_st = sum("scratch_store" in l for l in lines)
    tot_ld = sum("scratch_load" in l for l in lines)
    print(f"{name[11:70]}: scratch st {tot_st} ld {tot_ld}, {len(lines)} lines")
    for a, b in sorted(loops, key=lambda x: x[0] - x[1])[:3]:
        seg = lines[a:b]
        print(f"   loop {a}-{b} ({b - a} lines): st {sum('scratch_store' in l for l in seg)} "
              f"ld {sum('scratch_load' in l for l in seg)}")
