#!/usr/bin/env python3
"""Build timing-only variants of the kernel library for A/B runs (tools/ab_run.sh, prof_rollout
--lib): the product sources are copied to a scratch directory, one named text substitution set is
applied (each `old` must occur exactly once), and the copy is built into ab/lib_<variant>.so.  The
product sources carry no diagnostic switches; variants that cut work give WRONG answers and exist
only to locate time (never loaded by tests, smoke or bench).

    python tools/ab_variants.py <variant> [<variant> ...]      (list: python tools/ab_variants.py)
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "sparc-gym_amd", "csrc")

VARIANTS = {
    # the in-tree sources, built the same way (the A/B baseline)
    "head": [],
    # k_rollout1r audit waves: region codes not looked up (a constant code instead of reg_tab)
    "notab": [("sparc_rules.hpp", "            tw = rt.reg_tab[(fo + m) >> 3];", "            tw = 0x55555555u;")],
    # k_rollout1r audit waves: the puzzle's rule data loaded once, not on every puzzle change
    "noreload": [("sparc_kernels.hip", "                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);",
                  "                if (pr.q == 0xFFFFFFFFu) pr = puzzle_rules<1>(p, rt, pid);")],
    # the audit's flood fill cut to one dilation per region
    "noflood": [("sparc_rules.hpp", "            if (N == R) break;\n            R = N;", "            R = N;\n            break;")],
    # k_rollout1r audit waves do no audit at all (the step wave, rings and barriers only)
    "noaudit": [("sparc_kernels.hip", "            if (active) {\n                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);",
                 "            if (false) {\n                if (pid != pr.q) pr = puzzle_rules<1>(p, rt, pid);")],
    # c3 trie wave (TrieLane::step_core): the next reset's row read inside the reset branch into
    # the same registers (uses pinned ahead of it), not on every step
    "trienx": [("sparc_trie.hpp", """            tmax = nx.w >> 17;
        }
        // the row of the next reset, read every step outside the branch: read inside it, the
        // compiler lands it in temporaries and waits for it right there to copy it into nx
        nx = trow[npid];""", """            tmax = nx.w >> 17;
            __asm__ volatile("" ::: "memory");
            nx = trow[npid];
        }""")],
}


def build(name, jobs_dir):
    d = os.path.join(jobs_dir, name)
    shutil.copytree(CSRC, d)
    for fname, old, new in VARIANTS[name]:
        path = os.path.join(d, fname)
        src = open(path).read()
        if src.count(old) != 1:
            raise SystemExit(f"variant {name}: {old!r} occurs {src.count(old)} times in {fname}")
        open(path, "w").write(src.replace(old, new))
    out = os.path.join(REPO, "ab", f"lib_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(REPO, "include"), "-I" + d, "-o", out, os.path.join(d, "sparc_kernels.hip")]
    return subprocess.Popen(cmd), out


def main():
    names = sys.argv[1:]
    if not names:
        print("variants:", ", ".join(VARIANTS))
        return
    with tempfile.TemporaryDirectory() as tmp:
        procs = [build(n, tmp) for n in names]
        rc = 0
        for p, out in procs:
            rc |= p.wait()
            print(out, "ok" if p.returncode == 0 else f"FAILED ({p.returncode})")
    sys.exit(rc)


if __name__ == "__main__":
    main()
