"""bench.py --gpus N without torchrun: the parent starts one rank process per GPU itself.

The launcher (bench.launch_ranks) is host logic: these CPU tests run it on a tiny child script
instead of the bench, checking the rank environment it hands out and that a failing rank ends
the job with its exit code (the other ranks terminated, none left waiting in a collective).
"""
import json
import os
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

CHILD = r"""
import json, os, sys, time
out = sys.argv[1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "SPARC_BENCH_LAUNCHER")
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
if len(sys.argv) > 2 and os.environ["RANK"] == sys.argv[2]:
    sys.exit(3)
if len(sys.argv) > 3:
    time.sleep(float(sys.argv[3]))
"""


def _child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return [sys.executable, str(p)]


def test_launch_ranks_environment(tmp_path):
    rc = bench.launch_ranks(3, _child(tmp_path) + [str(tmp_path)], {"SPARC_BENCH_LAUNCHER": "1"})
    assert rc == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]   # one GPU per rank
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert {e["SPARC_BENCH_LAUNCHER"] for e in envs} == {"1"}


def test_launch_ranks_failing_rank_ends_job(tmp_path):
    t0 = time.time()
    # rank 1 fails at once; the others would sleep 60 s
    rc = bench.launch_ranks(3, _child(tmp_path) + [str(tmp_path), "1", "60"])
    assert rc == 3
    assert time.time() - t0 < 30


def test_world_mismatch_refused(monkeypatch):
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero before touching the GPU."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=2" in str(e.value)


def test_cpu_bench_covers_every_bench_config():
    """The multi-core CPU baseline (oracle/cpu_bench.py, run by bench's cpu_baseline leg) knows
    every bench workload with the same lattices, property set and traceback flag."""
    from oracle import cpu_bench
    for name, (sizes, full, tb, _obs) in bench.CONFIGS.items():
        assert cpu_bench.CONFIGS[name] == (sizes, full, tb), name


def test_rule_config_refuses_step_mode(monkeypatch, capsys):
    """--mode step runs no rule audit, so a rule config (c3r) in step mode is an argument error,
    not a line that labels a workload it never ran."""
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "c3r", "--mode", "step"])
    with pytest.raises(SystemExit) as e:
        bench.parse()
    assert e.value.code == 2
    assert "c3r" in capsys.readouterr().err


def test_cpu_baseline_cores_follow_the_job():
    """rank 0 times the CPU step() after the timed region at every world size,
    on the job's share of the host: 16 cores per GPU the job drives, at most the usable cores."""
    assert bench.cpu_procs(1, usable=8) == 8
    assert bench.cpu_procs(1, usable=256) == 16
    assert bench.cpu_procs(2, usable=256) == 32
    assert bench.cpu_procs(8, usable=256) == 128
    assert bench.cpu_procs(8, usable=64) == 64


def test_cpu_baseline_names_its_cores():
    """The C-oracle baseline leg on a small sample with two processes: the record names the
    processes it ran (cores) and the single-thread rate beside them."""
    import os as _os
    _os.environ["SPARC_POOL_WORKERS"] = "1"
    proc = bench.make_pool(64, ((3, 3),), True)
    cb = bench.cpu_baseline(proc, True, 2000, 0.5, None, "c3", procs=2)
    assert cb["cores"] == 2 and cb["value"] > 0 and cb["value_1core"] > 0
    assert "2 processes" in cb["sample"]
