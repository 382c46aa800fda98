#!/usr/bin/env python3
"""Compares the kernel bodies of two `make asm` outputs (build/mj423_kernels-gfx950.s):
per kernel symbol, identical or the changed instruction lines.  Used to show that a source
refactor leaves the production kernels' ISA unchanged.  usage: isa_diff.py BEFORE.s AFTER.s"""
import difflib
import re
import sys


def kernels(path):
    out, cur = {}, None
    for line in open(path).read().split("\n"):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur:
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            out[cur].append(line)
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            print(("NEW  " if k not in a else "GONE ") + k)
            continue
        if a[k] == b[k]:
            print(f"same {len(a[k]):5d} lines  {k}")
            continue
        d = [l for l in difflib.unified_diff(a[k], b[k], lineterm="", n=0)
             if l[:1] in "+-" and not l.startswith(("+++", "---"))]
        print(f"DIFF {len(d):5d} lines  {k}")
        for l in d[:12]:
            print("      " + l.strip())


if __name__ == "__main__":
    main()
