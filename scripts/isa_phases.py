"""Per-phase static instruction counts of one kernel compiled with -DTHESIA_MARKS
(asm comments "; MARK <phase>" at phase boundaries; basic blocks listed inside a phase).

usage: python scripts/isa_phases.py file.s KERNEL_SUBSTRING [min_valu]
"""
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    minv = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    text = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(sub) + r"\S*):\s*;\s*@", text, re.M)
    # to the function's end (an early return puts an s_endpgm in the middle of the body)
    body = text[m.end():text.find(".Lfunc_end", m.end())]
    cur, order, cnt = "entry", ["entry"], {}
    for line in body.split("\n"):
        t = line.strip()
        mk = re.search(r"MARK (\w+)", t)
        if mk:
            cur = mk.group(1)
            order.append(cur)
            continue
        if t.startswith(".LBB"):
            cur = cur.split("|")[0] + "|" + t.split(":")[0]
            order.append(cur)
            continue
        if not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        c = cnt.setdefault(cur, dict(valu=0, lds=0, salu=0, vmem=0, wait=0))
        if op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("s_waitcnt"):
            c["wait"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith(("global_", "buffer_", "scratch_")):
            c["vmem"] += 1
    for k in order:
        if k in cnt and cnt[k]["valu"] >= minv:
            print(f"{k:40s} {cnt[k]}")


if __name__ == "__main__":
    main()
