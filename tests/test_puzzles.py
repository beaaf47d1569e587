"""Host loader (restated _process_puzzles) and table packer, against the reference's output."""
import numpy as np
import pytest

import golden_io
from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import build_trie, lattice_geometry, pack_table, process_puzzles

DIRS = ((1, 0), (0, -1), (-1, 0), (0, 1))


@pytest.mark.parametrize("pool", golden_io.POOLS)
def test_process_puzzles_matches_reference(pool):
    g = golden_io.load(pool)
    mine = process_puzzles(g["records"])
    assert len(mine) == len(g["processed"])
    for m, r in zip(mine, g["processed"]):
        assert m["id"] == r["id"]
        assert (m["x_size"], m["y_size"]) == (r["x_size"], r["y_size"])
        assert list(m["start_location"]) == r["start"] and list(m["target_location"]) == r["target"]
        assert m["solution_count"] == r["solution_count"]
        assert m["solution_paths"] == r["solution_paths"]
        # key set AND order, including stale-`symbol` planes (SPaRC_Gym.py:283-343)
        assert list(m["obs_array"].keys()) == r["base_keys"]
        for k in r["base_keys"]:
            if k in ("visited", "agent_location", "target_location"):
                continue   # set by _load_puzzle, checked through the env tests
            assert np.array_equal(m["obs_array"][k], golden_io.dense(r["base"][k])), k
            assert m["obs_array"][k].dtype == np.int32
        assert np.array_equal(m["color_array"], golden_io.dense(r["color"]))
        assert np.array_equal(m["additional_info"], golden_io.dense(r["additional_info"]))
        assert m["additional_info"].dtype == np.int64


def test_unbound_symbol_raises_like_reference():
    g = golden_io.load("unbound_symbol")
    assert g["raises"] == "UnboundLocalError"
    with pytest.raises(UnboundLocalError):
        process_puzzles(g["records"])


def test_dataframe_and_records_agree():
    recs = synthetic.make_puzzles(5, seed=9)
    a = process_puzzles(recs)
    b = process_puzzles(synthetic.records_to_dataframe(recs))
    for x, y in zip(a, b):
        assert list(x["obs_array"]) == list(y["obs_array"])
        for k in x["obs_array"]:
            assert np.array_equal(x["obs_array"][k], y["obs_array"][k])


def _walk_trie(nodes, start, path):
    """trie walk: returns node index or None if the path leaves the trie."""
    cur = 0
    for (ax, ay), (bx, by) in zip(path[:-1], path[1:]):
        d = DIRS.index((bx - ax, by - ay))
        cur = nodes[cur][d]
        if cur == 0xFFFF:
            return None
    return cur


def _is_prefix(path, sols):
    return any(len(path) <= len(s) and all(path[i] == s[i] for i in range(len(path))) for s in sols)


@pytest.mark.parametrize("seed", range(6))
def test_trie_equals_list_compare(seed):
    """The trie's (node, terminal) answers _is_on_solution_path / array_equal exactly."""
    rng = np.random.default_rng(seed)
    p = synthetic.make_puzzle(rng, 3, 3, n_solutions=int(rng.integers(1, 9)), shared_prefix_prob=0.8)
    proc = process_puzzles([p])[0]
    sols = [[tuple(pt) for pt in s] for s in proc["solution_paths"]]
    start = tuple(proc["start_location"])
    nodes, root_valid = build_trie(start, proc["solution_paths"])
    assert root_valid == any(s and s[0] == start for s in sols)
    # every prefix of every solution, plus random walks
    cands = [s[:k] for s in sols for k in range(1, len(s) + 1)]
    for _ in range(300):
        path = [start]
        for _ in range(int(rng.integers(0, 12))):
            dx, dy = DIRS[int(rng.integers(4))]
            nxt = (path[-1][0] + dx, path[-1][1] + dy)
            if nxt in path:
                break
            path.append(nxt)
        cands.append(path)
    for path in cands:
        node = _walk_trie(nodes, start, path) if root_valid else None
        assert (node is not None) == _is_prefix(path, sols)
        assert (node is not None and nodes[node][5] == 1) == (path in sols)


def test_pack_table_layout():
    recs = synthetic.make_puzzles(20, seed=3, sizes=((2, 2), (3, 3), (5, 5)))
    proc = process_puzzles(recs)
    t = pack_table(proc)
    assert (t.pitch, t.words, t.x_max, t.y_max) == (11, 2, 11, 11)
    for q, p in enumerate(proc):
        X, Y = p["x_size"], p["y_size"]
        info = t.info[q]
        assert (info[0] & 0xFF, (info[0] >> 8) & 0xFF) == (X, Y)
        gaps = p["obs_array"]["gaps"]
        for x in range(X):
            for y in range(Y):
                b = x * t.pitch + y
                bit = (int(t.open[q, b >> 6]) >> (b & 63)) & 1
                assert bit == (gaps[x, y] == 0)
        if info[1] >> 17 & 1:
            base, cnt = int(info[2]), int(info[3])
            assert cnt >= 1 and base + cnt <= len(t.trie)


def test_geometry_limits():
    assert lattice_geometry([{"x_size": 7, "y_size": 7}]) == (8, 1, 7, 7)      # padded
    assert lattice_geometry([{"x_size": 5, "y_size": 5}]) == (6, 1, 5, 5)
    assert lattice_geometry([{"x_size": 7, "y_size": 7}], words=2) == (7, 2, 7, 7)
    assert lattice_geometry([{"x_size": 7, "y_size": 9}]) == (9, 2, 7, 9)
    assert lattice_geometry([{"x_size": 11, "y_size": 11}]) == (11, 2, 11, 11)
    assert lattice_geometry([{"x_size": 15, "y_size": 15}]) == (15, 4, 15, 15)
    with pytest.raises(ValueError):
        lattice_geometry([{"x_size": 17, "y_size": 17}])
    with pytest.raises(ValueError):
        lattice_geometry([{"x_size": 7, "y_size": 7}], words=1, pitch=7)
    with pytest.raises(ValueError):
        lattice_geometry([{"x_size": 9, "y_size": 9}], words=1)
