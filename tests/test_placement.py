"""XCD-local first puzzles (sparc_gym_amd.vec_env.xcd_local_puzzle_index, bench.initial_puzzles):
a permutation of the plain hash placement's multiset of start puzzles over env slots, one eighth of
the pool per XCD group of 256-env workgroups (CPU only: host-side index arithmetic)."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sparc-gym_amd")]


@pytest.mark.parametrize("P", [2048, 4096, 16384])
@pytest.mark.parametrize("offset", [0, 65536])
def test_xcd_local_start_puzzles(P, offset):
    from sparc_gym_amd.vec_env import xcd_local_puzzle_index
    n = 65536
    q = xcd_local_puzzle_index(n, P, offset)
    assert q.dtype == np.int64 and q.shape == (n,) and q.min() >= 0 and q.max() < P
    # every puzzle starts the same number of envs, as with env i -> i * 2654435761 mod P
    assert np.all(np.bincount(q, minlength=P) == n // P)
    # workgroup b (256 envs) runs on XCD group b % 8 and starts only on block b % 8 of the pool
    blk = (q // (P // 8)).reshape(-1, 256)
    assert np.all(blk == (np.arange(n // 256) % 8)[:, None])
    # the envs of one workgroup do not share a start puzzle
    assert all(len(set(r)) == 256 for r in q.reshape(-1, 256).tolist()) if P // 8 >= 256 else True


def test_bench_placement_auto():
    import bench
    gid = np.arange(65536, dtype=np.uint64)
    for P, want in ((1024, "hash"), (4096, "xcd"), (16384, "xcd"), (1000, "hash")):
        q, used = bench.initial_puzzles(gid, P, "auto")
        assert used == want and q.min() >= 0 and q.max() < P
    q, used = bench.initial_puzzles(gid, 16384, "hash")
    assert used == "hash" and np.array_equal(q, (gid * np.uint64(2654435761) % np.uint64(16384)).astype(np.int64))


def test_small_or_odd_pools_fall_back_to_the_hash():
    from sparc_gym_amd.vec_env import xcd_local_puzzle_index
    for P in (1, 5, 1001):
        q = xcd_local_puzzle_index(4096, P)
        assert np.array_equal(q, (np.arange(4096, dtype=np.uint64) * np.uint64(2654435761) % np.uint64(P)).astype(np.int64))
