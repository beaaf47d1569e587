#!/usr/bin/env python3
"""Per-role cycle stamps of k_rollout1r (the c3r kernel) from the `stamps` build of
tools/ab_variants.py: for the step waves and the audit waves, the mean cycles per launch in
total, waiting at the tile barriers and (audit waves) inside their audits (s_memtime).

    python tools/ab_variants.py stamps && python tools/diag_r1r.py [--chunk 50]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from sparc_gym_amd import _lib  # noqa: E402

_lib.load(os.path.join(REPO, "ab", "lib_stamps.so"))
import bench  # noqa: E402
from sparc_gym_amd import SPaRCVecEnv, synthetic  # noqa: E402
from sparc_gym_amd.puzzles import process_puzzles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chunk", type=int, default=50)
ap.add_argument("--envs", type=int, default=65536)
a = ap.parse_args()
sizes, full, tb, _ = bench.CONFIGS["c3r"]
proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=sizes, full_properties=full))
vec = SPaRCVecEnv(a.envs, processed=proc, traceback=tb, observation="compact", rules=True)
gid = np.arange(a.envs, dtype=np.uint64)
vec.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})
vec._stream()
T, n = a.chunk, a.envs
rew = torch.empty((T, n), dtype=torch.int8, device="cuda")
flg = torch.empty((T, n), dtype=torch.uint8, device="cuda")
bits = torch.empty((T, n), dtype=torch.int16, device="cuda")
for k in range(4):
    acts = vec.random_actions(T, seed=9, t0=k * T)
    st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    vec.core.rollout_rules_device(T, acts.data_ptr(), rew.data_ptr(), flg.data_ptr(), st.data_ptr(), bits.data_ptr())
    torch.cuda.synchronize()
d = st.cpu().numpy()[n // 2:]
d = d[d[:, 1] > 0]
for role, name in ((0, "step waves"), (1, "audit waves")):
    r = d[d[:, 0] == 0] if role == 0 else d[d[:, 0] > 0]
    print(f"{name}: {len(r)} waves, total {r[:, 1].mean():.0f} cycles, barrier wait {r[:, 2].mean():.0f}"
          + (f", in audits {r[:, 3].mean():.0f} (max {r[:, 3].max()})" if role else ""))
print(f"T = {T}: per step {d[:, 1].mean() / T:.0f} cycles")
