"""Instruction histogram of one kernel in a hipcc -S output (static counts; loops not weighted).

usage: python scripts/isa_hist.py file.s SUBSTRING [top]
"""
import collections
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", text, re.M):
        name = m.group(1)
        end = text.find("s_endpgm", m.end())
        yield name, text[m.end():end]


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    text = open(path).read()
    for name, body in kernels(text):
        if sub not in name:
            continue
        c = collections.Counter()
        for line in body.split("\n"):
            line = line.strip()
            if not line or line.startswith((".", ";")) or line.endswith(":"):
                continue
            c[line.split()[0]] += 1
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{name}: {sum(c.values())} instrs, {valu} VALU")
        m = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", text)
        if m:
            print("  vgpr", m.group(1))
        for k, v in c.most_common(top):
            print(f"  {v:6d} {k}")


if __name__ == "__main__":
    main()
