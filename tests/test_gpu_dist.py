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


def _bench_cmd(*extra, cpu=False):
    return [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"),
            *(["--cpu-seconds", "1"] if cpu else ["--no-cpu-baseline"]),
            "--steps", "2", "--warmup", "1", "--env-steps", "64", "--envs", "4096"] + list(extra)


def test_bench_gpus2_launches_two_ranks_itself(on_gpu):
    """`python bench.py --gpus 2` (no torchrun) starts two rank processes itself; on the box's
    one GPU that is a rehearsal (gloo, both ranks on GPU 0), and the JSON line reports the
    world the ranks observed."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(_bench_cmd("--gpus", "2", "--rehearsal", "--backend", "gloo", cpu=True), env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                          # rank 0 prints one line
    o = json.loads(lines[0])
    w = o["world_observed"]
    assert o["n_gpus"] == 2 and w["world_size"] == 2 and w["backend"] == "gloo"
    assert w["launcher"] == "bench.py (child per rank)" and w["rehearsal"] is True
    assert len(w["per_rank_kernel_ms"]) == 2 and all(t > 0 for t in w["per_rank_kernel_ms"])
    assert o["episodes"]["done"] > 0
    assert o["value"] > 0
    # the CPU step() beside the GPU number at world 2 too (rank 0, after the timed region), on the
    # job's share of the host: the one GPU both ranks drive -> at most 16 cores
    cb = o["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and 1 <= cb["cores"] <= 16, cb


def test_bench_refuses_two_ranks_on_one_gpu(on_gpu):
    """Without --rehearsal, more ranks than GPUs is an error (non-zero exit), not a number."""
    if torch.cuda.device_count() != 1:
        pytest.skip("needs a one-GPU box")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(_bench_cmd("--gpus", "2", "--backend", "gloo"), env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_rccl_paths_at_world_one(on_gpu, tmp_path):
    """torch.distributed over RCCL ("nccl") and the C-ABI's own RCCL gather, on the one GPU."""
    import json
    out = str(tmp_path / "rccl.json")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_rccl_worker.py"), out], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    got = json.load(open(out))
    assert got["ok"] and got["backend"] == "nccl"
    assert got["torch_gather_equal"] and got["abi_gather_equal"]
    assert got["torch_values"] == [[1.5, 7.0]]
    assert got["bad_rank_rc"] == -1
