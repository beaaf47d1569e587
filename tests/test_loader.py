"""Local puzzle sources: a parquet export / json(l) of the SPaRC schema gives the
same processed puzzles as the in-memory records (the pinned `_process_puzzles` restatement)."""
import numpy as np
import pytest

from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import process_puzzles

pytest.importorskip("pyarrow")


def _same(a, b):
    assert len(a) == len(b)
    for p, q in zip(a, b):
        assert list(p["obs_array"]) == list(q["obs_array"])
        for k in p["obs_array"]:
            assert np.array_equal(p["obs_array"][k], q["obs_array"][k])
        for k in ("x_size", "y_size", "solution_count", "start_location", "target_location", "id", "difficulty",
                  "polyshapes"):
            assert p[k] == q[k], k
        assert [list(map(list, s)) for s in p["solution_paths"]] == [list(map(list, s)) for s in q["solution_paths"]]
        assert np.array_equal(p["color_array"], q["color_array"])
        assert np.array_equal(p["additional_info"], q["additional_info"])


@pytest.fixture(scope="module")
def records():
    return (synthetic.make_puzzles(12, seed=4, sizes=((2, 2), (3, 3), (5, 5)), full_properties=True)
            + synthetic.make_rule_puzzles(8, seed=5))


def test_parquet_file_and_directory(tmp_path, records):
    from sparc_gym_amd.env import load_puzzle_source
    df = synthetic.records_to_dataframe(records)
    f = tmp_path / "test-00000-of-00001.parquet"
    df.to_parquet(f)
    want = process_puzzles(records)
    _same(process_puzzles(load_puzzle_source(str(f), None, None, None)), want)
    d = tmp_path / "split"
    d.mkdir()
    df.iloc[:7].to_parquet(d / "a.parquet")
    df.iloc[7:].reset_index(drop=True).to_parquet(d / "b.parquet")
    _same(process_puzzles(load_puzzle_source(str(d), None, None, None)), want)


def test_jsonl(tmp_path, records):
    from sparc_gym_amd.env import load_puzzle_source
    f = tmp_path / "p.jsonl"
    synthetic.records_to_dataframe(records).to_json(f, orient="records", lines=True)
    _same(process_puzzles(load_puzzle_source(str(f), None, None, None)), process_puzzles(records))


def test_bad_path(tmp_path):
    from sparc_gym_amd.env import load_puzzle_source
    with pytest.raises(ValueError):
        load_puzzle_source(str(tmp_path), None, None, None)
