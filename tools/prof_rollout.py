#!/usr/bin/env python3
"""Fixed rollout workload for rocprofv3 counter passes (same setup as bench.py's default line):
65,536 envs, config c3, `--launches` rollout launches of `--chunk` env-steps each."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sparc-gym_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402  (no torch import at module level)

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--chunk", type=int, default=500)
ap.add_argument("--launches", type=int, default=4)
ap.add_argument("--rand", action="store_true", help="in-kernel counter-based actions (no action loads)")
ap.add_argument("--no-out", action="store_true", help="do not write reward codes / flags")
ap.add_argument("--time", action="store_true", help="print the mean launch time (HIP events)")
ap.add_argument("--lib", default=None, help="path of a diagnostic build of libsparc_gym_amd.so")
ap.add_argument("--rules", action="store_true", help="the rule audit after every step (rollout(rules=True))")
ap.add_argument("--puzzles", type=int, default=1024, help="pool size (bench.make_pool: blocks of 1,024)")
ap.add_argument("--placement", default="auto", choices=["auto", "hash", "xcd"], help="bench.initial_puzzles")
ap.add_argument("--variant", action="append", default=[],
                help="sparc_set_variant(ctx, VARIANT, 1), or VARIANT:VALUE, before the launches "
                     "(core.VARIANT_*; repeatable)")
a = ap.parse_args()
sizes, full, tb, obs = bench.CONFIGS[a.config]
proc = bench.make_pool(a.puzzles, sizes, full)   # before torch / any GPU call (worker processes fork)

import torch  # noqa: E402

if a.lib:   # another build of the library, loaded (after torch's HIP runtime) before the package uses it
    torch.cuda.init()
    from sparc_gym_amd import _lib as _sparc_lib  # noqa: E402
    _sparc_lib.load(os.path.abspath(a.lib), any_abi=True)

from sparc_gym_amd import SPaRCVecEnv  # noqa: E402
from sparc_gym_amd.puzzles import pack_table  # noqa: E402

a.rules = a.rules or a.config in bench.RULE_CONFIGS
table = pack_table(proc)
vec = SPaRCVecEnv(a.envs, processed=proc, table=table, traceback=tb, observation="compact", rules=a.rules)
for v in a.variant:
    which, _, value = v.partition(":")
    vec.core.set_variant(int(which), int(value or 1))
gid = np.arange(a.envs, dtype=np.uint64)
vec.reset(options={"puzzle_index": bench.initial_puzzles(gid, len(proc), a.placement)[0]})
acts = torch.randint(0, 4, (a.launches + 1, a.chunk, a.envs), dtype=torch.uint8, device="cuda")
rew = torch.empty((a.chunk, a.envs), dtype=torch.int8, device="cuda")
flg = torch.empty((a.chunk, a.envs), dtype=torch.uint8, device="cuda")
stats = torch.zeros((a.envs, 4), dtype=torch.int32, device="cuda")
ovis = oag = None
if obs:   # c4: 'new' observation traces [chunk, N, x_dim, y_dim] int32, as bench.py
    ovis = torch.empty((a.chunk, a.envs, vec.x_dim, vec.y_dim), dtype=torch.int32, device="cuda")
    oag = torch.empty_like(ovis)
bits = torch.empty((a.chunk, a.envs), dtype=torch.int16, device="cuda") if a.rules else None
if a.rules:
    vec._stream()
ms = []
for k in range(a.launches + 1):      # first launch = warmup
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if a.rules:   # the bench's direct C-ABI call (rollout(rules=True) would add a host sync per launch)
        vec.core.rollout_rules_device(a.chunk, None if a.rand else acts[k].data_ptr(), rew.data_ptr(), flg.data_ptr(),
                                      stats.data_ptr(), bits.data_ptr(), seed=k)
    elif a.no_out:
        vec.rollout(a.chunk, None if a.rand else acts[k], stats=stats, record=False, seed=k)
    else:
        vec.rollout(a.chunk, None if a.rand else acts[k], stats=stats, out=(rew, flg), seed=k,
                    obs_out=(ovis, oag) if obs else None)
    e1.record()
    ms.append((e0, e1))
torch.cuda.synchronize()
if a.time:
    t = [x.elapsed_time(y) for x, y in ms[1:]]
    print(f"rollout ms/launch {sum(t) / len(t):.4f}  env-steps/s {a.envs * a.chunk / (sum(t) / len(t) / 1e3):.4e}"
          f"  rand={a.rand} no_out={a.no_out}")
print("done", a.config, a.envs, a.chunk, a.launches)
