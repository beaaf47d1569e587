import sys, os
sys.path[:0] = ['/root/repo', '/root/repo/sparc-gym_amd', '/root/repo/tests']
import numpy as np, torch
from sparc_gym_amd import SPaRCVecEnv, synthetic
from sparc_gym_amd.puzzles import pack_table, process_puzzles
from test_gpu_parity import _make
proc, table = _make("7x7_full", seed=9)
def run(n, chunks, T=None):
    T = sum(chunks)
    pids = (np.arange(n) * 7) % len(proc)
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    acts = torch.randint(0, 5, (T, n), dtype=torch.uint8, device="cuda", generator=g)
    kw = dict(processed=proc, table=table, traceback=True, observation="compact", max_steps=60)
    a = SPaRCVecEnv(n, **kw); a.reset(options={"puzzle_index": pids})
    full = a.rollout(T, acts)
    b = SPaRCVecEnv(n, **kw); b.reset(options={"puzzle_index": pids})
    parts, t = [], 0
    for c in chunks:
        parts.append(b.rollout(c, acts[t:t + c].contiguous())); t += c
    r = []
    for key in ("reward_code", "flags"):
        x, y = full[key], torch.cat([p[key] for p in parts])
        bad = (x != y).nonzero()
        r.append((key, int(bad.shape[0]), bad[:5].tolist()))
    print(n, chunks, r, flush=True)
for n, ch in [(2048, (100, 57, 1, 32)), (2624, (96, 94)), (2624, (100, 90)), (2624, (1, 189)), (2624, (100, 57, 1, 32)), (2048, (190,)), (2624, (32, 158))]:
    run(n, ch)
