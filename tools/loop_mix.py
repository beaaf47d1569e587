#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a gfx950 .s file (make asm).

Usage: loop_mix.py <file.s> <kernel-symbol-substring> [--dump HEADER]
Per loop (every depth): VALU / SALU / LDS / VMEM / branch / wait / nop counts of the blocks the
compiler annotates as belonging to that loop ('in Loop: Header=...' comments; a nested loop's
blocks are counted under the innermost header only).  --dump prints that loop's blocks."""
import collections
import re
import sys


def kind(op):
    return ("LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_")) else
            "branch" if op.startswith("s_cbranch") or op == "s_branch" else "nop" if op == "s_nop" else
            "wait" if op.startswith("s_waitcnt") else "SALU" if op.startswith("s_") else
            "VALU" if op.startswith("v_") else "other")


def main():
    path, sym = sys.argv[1:3]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(sym), l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    loops = collections.OrderedDict()
    cur = None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?\s*(;.*)?$", l)
        if m:
            c = m.group(2) or ""
            h = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", c)
            d = re.search(r"Loop Header: Depth=(\d+)", c)
            if d:
                cur = (m.group(1).lstrip(".L"), d.group(1))
            elif h:
                cur = (h.group(1), h.group(2))
            else:
                cur = None
            if dump and cur and cur[0] == dump:
                print(l)
            continue
        if cur is None:
            continue
        if dump and cur[0] == dump:
            print(l)
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        loops.setdefault(cur, collections.Counter())[kind(t[0])] += 1
    if not dump:
        for (hdr, depth), c in loops.items():
            print(f"{hdr} depth {depth} {dict(c)} total {sum(c.values())}")


if __name__ == "__main__":
    main()
