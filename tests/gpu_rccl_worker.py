"""The product's RCCL paths on one GPU, as a rank of a world of one (tests/test_gpu_dist.py runs it).

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so this
exercises every RCCL call the multi-GPU bench makes, at world size 1:
  * torch.distributed with backend "nccl" (= RCCL): sparc_gym_amd.dist.gather_stats
    (all_gather_into_tensor of the device stats) and gather_values;
  * the C-ABI gather (sparc_comm_unique_id / sparc_comm_init / sparc_gather_stats, librccl
    through the HIP library, no torch in the call) after a HIP rollout.
Writes a JSON verdict to argv[1].

    MASTER_ADDR=127.0.0.1 MASTER_PORT=... python tests/gpu_rccl_worker.py OUT.json
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "sparc-gym_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sparc_gym_amd import SPaRCVecEnv, _lib, synthetic  # noqa: E402
from sparc_gym_amd import dist as sdist  # noqa: E402
from sparc_gym_amd.puzzles import pack_table, process_puzzles  # noqa: E402


def main():
    out = {}
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    proc = process_puzzles(synthetic.make_puzzles(64, seed=3, sizes=((3, 3),), full_properties=True))
    table = pack_table(proc)
    n, T = 4096, 64
    v = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, observation="compact", device=0)
    v.reset(options={"puzzle_index": np.arange(n) % len(proc)})
    stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    v.rollout(T, None, seed=5, stats=stats)
    torch.cuda.synchronize()
    assert int(stats[:, 1].sum()) > 0
    # --- torch.distributed over RCCL, world 1
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out["backend"] = dist.get_backend()
    g = sdist.gather_stats(stats)
    torch.cuda.synchronize()
    out["torch_gather_equal"] = bool(g.device == stats.device and torch.equal(g, stats) and g.data_ptr() != stats.data_ptr())
    out["torch_values"] = sdist.gather_values([1.5, 7], dev)
    dist.destroy_process_group()
    # --- the C ABI's own RCCL communicator (no torch in the collective)
    lib = _lib.load()
    uid = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(lib.sparc_comm_unique_id(uid))
    comm = ctypes.c_void_p()
    _lib.check(lib.sparc_comm_init(v.core.ctx, 1, 0, uid, ctypes.byref(comm)), v.core.ctx)
    assert comm.value
    # bad rank is refused before RCCL
    bad = ctypes.c_void_p()
    out["bad_rank_rc"] = lib.sparc_comm_init(v.core.ctx, 1, 1, uid, ctypes.byref(bad))
    v._stream()
    gathered = torch.full((n, 4), -7, dtype=torch.int32, device=dev)
    _lib.check(lib.sparc_gather_stats(v.core.ctx, comm, stats.data_ptr(), gathered.data_ptr()), v.core.ctx)
    v.core.sync()
    out["abi_gather_equal"] = bool(torch.equal(gathered, stats))
    _lib.check(lib.sparc_comm_destroy(comm))
    out["ok"] = True
    with open(sys.argv[1], "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
