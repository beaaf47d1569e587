#!/usr/bin/env python3
"""Wall time per SPaRCVecEnv.step() call (the gym one-call-per-step contract) at 65,536 c3 envs.

Times `--calls` back-to-back calls after a warm-up, synchronised once at the end, for actions
given as a CUDA int64 tensor and as a numpy int64 array, with observation 'new' and 'compact'.
`legacy` reproduces the previous composition for comparison: the step_obs launch followed by
separate torch launches for the float64 reward, the bool flags, the info fields and agent_xy."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sparc_gym_amd import SPaRCVecEnv, synthetic  # noqa: E402
from sparc_gym_amd.puzzles import pack_table, process_puzzles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--calls", type=int, default=300)
a = ap.parse_args()
sizes, full, tb, _ = bench.CONFIGS["c3"]
proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=sizes, full_properties=full))
table = pack_table(proc)


def legacy_step(v, act_u8):
    """The pre-fused SPaRCVecEnv.step body (uint8 actions already on the device)."""
    v._act.copy_(act_u8)
    new = v.observation == "new"
    v.core.step_obs_device(v._act.data_ptr(), v._rew.data_ptr(), v._flags.data_ptr(),
                           v._vis.data_ptr() if new else None, v._agent.data_ptr() if new else None,
                           v.x_dim if new else 1, v.y_dim if new else 1, v._pidx.data_ptr(), v._pos.data_ptr())
    f = v._flags
    reward = v._rew.to(torch.float64) / 100.0
    info = {"legal_mask": (f >> 2) & 0xF, "autoreset": (f & 64).bool(), "reward_code": v._rew}
    return v._obs_dict(), reward, (f & 1).bool(), (f & 2).bool(), info


for obs in ("new", "compact"):
    v = SPaRCVecEnv(a.envs, processed=proc, table=table, traceback=tb, observation=obs)
    v.reset(seed=0)
    rng = np.random.default_rng(0)
    host = [rng.integers(0, 4, a.envs).astype(np.int64) for _ in range(8)]
    dev64 = [torch.from_numpy(h).cuda() for h in host]
    dev8 = [d.to(torch.uint8) for d in dev64]
    cases = {"cuda_int64": lambda k: v.step(dev64[k % 8]),
             "numpy_int64": lambda k: v.step(host[k % 8]),
             "legacy_cuda_uint8": lambda k: legacy_step(v, dev8[k % 8])}
    for name, fn in cases.items():
        for k in range(20):
            fn(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.calls):
            fn(k)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.calls * 1e6
        print(f"obs={obs:8s} {name:18s} {us:8.1f} us per step() call, {a.envs / us * 1e6:.3e} env-steps/s",
              flush=True)
