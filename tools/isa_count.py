"""Instruction classes of one kernel in a hipcc -S listing, per basic block (measurement only).
  python tools/isa_count.py listing.s KERNEL_SUBSTRING [--blocks]"""
import re
import sys


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_nop", "s_setprio", "s_sleep", "s_endpgm")):
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if re.match(r"^_ZN\S*" + re.escape(key) + r"\S*:", l))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], {}, "entry"
    for l in lines[st + 1:en]:
        t = l.strip()
        if re.match(r"^\.LBB\S*:", t):
            blocks.append((name, cur))
            name, cur = t.split(":")[0], {}
            continue
        if not t or t.startswith((".", ";")):
            continue
        c = classify(t.split()[0])
        if c:
            cur[c] = cur.get(c, 0) + 1
        if t.startswith("s_cbranch") or t.startswith("s_branch"):
            cur.setdefault("->", []).append(t.split()[-1])
    blocks.append((name, cur))
    tot = {}
    for _, c in blocks:
        for k, v in c.items():
            if k != "->":
                tot[k] = tot.get(k, 0) + v
    print(lines[st].split(":")[0][:100], tot)
    if "--blocks" in sys.argv:
        for n, c in blocks:
            print(f"  {n:12s} " + " ".join(f"{k}={v}" for k, v in c.items()))


if __name__ == "__main__":
    main()
