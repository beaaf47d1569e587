#!/usr/bin/env python3
"""Time the rule audit (k_rules) on the bench workload: c3 pool, 65,536 envs, after a device
rollout of --warm random steps (so paths have split the boards into regions)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

if "--lib" in sys.argv:   # another build of the library, loaded before the package uses it
    from sparc_gym_amd import _lib as _sparc_lib  # noqa: E402
    _sparc_lib.load(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sparc_gym_amd import SPaRCVecEnv, synthetic  # noqa: E402
from sparc_gym_amd.puzzles import pack_table, process_puzzles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--warm", type=int, default=20)
ap.add_argument("--launches", type=int, default=10)
ap.add_argument("--rule-pool", action="store_true", help="rule-consistent puzzles instead of the bench pool")
ap.add_argument("--lib", default=None, help="path of a diagnostic build of libsparc_gym_amd.so")
a = ap.parse_args()
sizes, full, tb, obs = bench.CONFIGS[a.config]
recs = (synthetic.make_rule_puzzles(1024, seed=0, sizes=sizes) if a.rule_pool
        else synthetic.make_puzzles(1024, seed=0, sizes=sizes, full_properties=full))
proc = process_puzzles(recs)
vec = SPaRCVecEnv(a.envs, processed=proc, table=pack_table(proc), traceback=tb, observation="compact", rules=True)
gid = np.arange(a.envs, dtype=np.uint64)
vec.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})
vec.rollout(a.warm, None, seed=1, record=False)
vec.rule_audit()
torch.cuda.synchronize()
ev = []
for k in range(a.launches):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = vec.rule_audit()
    e1.record()
    ev.append((e0, e1))
torch.cuda.synchronize()
vec.core.sync()
ms = float(np.mean([x.elapsed_time(y) for x, y in ev]))
bits = r["bits"].cpu().numpy().astype(np.uint16)
print(f"rules {a.config} envs={a.envs} warm={a.warm}: {ms:.4f} ms/launch, {a.envs / ms * 1e3:.4e} audits/s; "
      f"pass rates " + " ".join(f"{(bits >> k & 1).mean():.3f}" for k in range(9)))
