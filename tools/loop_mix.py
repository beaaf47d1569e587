#!/usr/bin/env python3
"""Instruction mix of the innermost loops of one kernel in a gfx950 .s file (make asm).

Usage: loop_mix.py <file.s> <kernel-symbol-substring>
Per depth-2 loop: VALU / SALU / LDS / VMEM / branch / nop counts of every block the compiler
annotates as belonging to that loop (the 'in Loop: Header=...' comments)."""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1:3]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(sym), l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    loops = collections.OrderedDict()
    cur = None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?\s*(;.*)?$", l)
        if m:
            c = m.group(2) or ""
            h = re.search(r"Header=(BB\d+_\d+) Depth=2", c)
            if "Inner Loop Header: Depth=2" in c:
                cur = m.group(1).lstrip(".L")
            elif h:
                cur = h.group(1)
            else:
                cur = None
            continue
        if cur is None:
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        op = t[0]
        k = ("LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_")) else
             "branch" if op.startswith("s_cbranch") or op == "s_branch" else "nop" if op == "s_nop" else
             "wait" if op.startswith("s_waitcnt") else "SALU" if op.startswith("s_") else
             "VALU" if op.startswith("v_") else "other")
        loops.setdefault(cur, collections.Counter())[k] += 1
    for h, c in loops.items():
        print(h, dict(c), "total", sum(v for k, v in c.items() if k not in ("wait", "nop")))


if __name__ == "__main__":
    main()
