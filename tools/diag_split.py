#!/usr/bin/env python3
"""Per-role timing of the W = 1 split rollout (tools/diag/libsparc_diag.so: k_rollout1s with
s_memtime stamps).  Same workload as bench.py / prof_rollout.py; prints, per role (move, trie,
I/O wave), the mean cycles per tile interval spent working and waiting at the tile barrier, and
the cycles per env-step.  The stamps themselves cost a little (guide: ~+11 % wave cycles)."""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from sparc_gym_amd import _lib  # noqa: E402

_name = sys.argv[sys.argv.index("--diag-lib") + 1] if "--diag-lib" in sys.argv else "libsparc_diag.so"
lib = _lib.load(os.path.join(REPO, "tools", "diag", _name))
lib.sparc_diag_rollout1s.argtypes = [ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 5 + [ctypes.c_int32]
lib.sparc_diag_rollout1s.restype = ctypes.c_int32

import bench  # noqa: E402
from sparc_gym_amd import SPaRCVecEnv, synthetic  # noqa: E402
from sparc_gym_amd.puzzles import pack_table, process_puzzles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--chunk", type=int, default=2000)
ap.add_argument("--launches", type=int, default=4)
ap.add_argument("--diag-lib", default="libsparc_diag.so")
ap.add_argument("--variant", type=int, default=0, help="trie gather: 0 global (product), 1 LDS (fake records), 2 none")
ap.add_argument("--puzzles", type=int, default=1024, help="pool size (bench.make_pool); past 1,024 the global-row kernel")
a = ap.parse_args()
sizes, full, tb, obs = bench.CONFIGS[a.config]
proc = (process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=sizes, full_properties=full)) if a.puzzles == 1024
        else bench.make_pool(a.puzzles, sizes, full))
table = pack_table(proc)
vec = SPaRCVecEnv(a.envs, processed=proc, table=table, traceback=tb, observation="compact")
gid = np.arange(a.envs, dtype=np.uint64)
vec.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})
vec._stream()
acts = torch.randint(0, 4, (a.chunk, a.envs), dtype=torch.uint8, device="cuda")
rew = torch.empty((a.chunk, a.envs), dtype=torch.int8, device="cuda")
flg = torch.empty((a.chunk, a.envs), dtype=torch.uint8, device="cuda")
stats = torch.zeros((a.envs, 4), dtype=torch.int32, device="cuda")
blocks = a.envs // 256
times = torch.zeros((blocks, 12, 4), dtype=torch.int64, device="cuda")
ms = []
for k in range(a.launches + 1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.check(lib.sparc_diag_rollout1s(vec.core.ctx, a.chunk, acts.data_ptr(), rew.data_ptr(), flg.data_ptr(),
                                        stats.data_ptr(), times.data_ptr(), a.variant), vec.core.ctx)
    e1.record()
    ms.append((e0, e1))
torch.cuda.synchronize()
t = times.cpu().numpy().astype(np.float64)          # the last launch
kern = float(np.mean([x.elapsed_time(y) for x, y in ms[1:]]))
print(f"diag kernel ms/launch {kern:.4f} ({a.config}, {a.envs} envs, {a.chunk} steps, variant {a.variant})")
for name, sl in (("move", slice(0, 4)), ("trie", slice(4, 8)), ("io", slice(8, 12))):
    r = t[:, sl, :].reshape(-1, 4)
    tiles = r[:, 3].mean()
    print(f"{name:5s} work/tile {r[:, 0].mean() / tiles:9.1f}  barrier/tile {r[:, 1].mean() / tiles:9.1f}  "
          f"all {r[:, 2].mean():12.0f} cyc  per env-step: work {r[:, 0].mean() / a.chunk:7.1f} "
          f"barrier {r[:, 1].mean() / a.chunk:7.1f}  (tiles {tiles:.0f}; work p10/p90 per tile "
          f"{np.percentile(r[:, 0] / r[:, 3], 10):.0f}/{np.percentile(r[:, 0] / r[:, 3], 90):.0f})")
