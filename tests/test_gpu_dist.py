"""Multi-GPU path with the HIP kernels in every rank (BASELINE config c5 shape per rank).

Two ranks (torchrun, gloo, both on the box's one GPU) each run the HIP rollout on their shard
of 65,536 envs (tests/gpu_dist_worker.py); the all_gathered per-env stats and the gathered
reward-code / flag traces must equal ONE process running the HIP rollout over all 131,072 envs.
The ranks are separate processes started through torchrun (subprocess); this test process only
compares."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_hip_rollout_equals_single_process(on_gpu, tmp_path):
    n, T, seed = 65536, 96, 31
    out = str(tmp_path / "dist.npz")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "gpu_dist_worker.py"), out, "--envs", str(n), "--steps", str(T), "--seed", str(seed)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    got = np.load(out)
    assert int(got["world"]) == 2 and str(got["backend"]) == "gloo"
    assert float(got["elapsed"]) == pytest.approx(1.5)               # max over ranks
    sys.path.insert(0, HERE)
    from gpu_dist_worker import pool, run_envs
    proc, table = pool()
    stats, rew, flg = run_envs(proc, table, 0, 2 * n, T, seed)
    assert np.array_equal(got["stats"], stats.cpu().numpy())
    assert np.array_equal(got["reward"], rew.cpu().numpy())
    assert np.array_equal(got["flags"], flg.cpu().numpy())
    assert int(got["stats"][:, 1].sum()) > 0                         # episodes ended in both shards
    assert got["stats"][:n, 1].sum() > 0 and got["stats"][n:, 1].sum() > 0
