"""The C rule-audit port (oracle/sparc_rules_oracle.c, the c3r CPU baseline's audit) against the
reference's own rule_status bits (tests/golden/rules_*.json.gz) and against oracle/rules_ref.py on
random walks over the bench's c3r pool."""
import os
import sys

import numpy as np
import pytest

from golden_io import load
from oracle import RulesCOracle, rules_ref
from rules_io import RULE_POOLS, ref_puzzle, snapshots

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("pool", RULE_POOLS)
def test_c_rules_match_reference_bits(pool):
    g = load(pool)
    puzzles = [ref_puzzle(p) for p in g["processed"]]
    co = RulesCOracle(puzzles)
    n = 0
    for e, pi, t, s in snapshots(g):
        assert co.bits(pi, s["path"], s["agent"]) == rules_ref.rule_bits(s["rule_status"]), (pool, e, t)
        n += 1
    assert n > 50


def test_c_rules_match_python_port_on_bench_pool():
    sys.path[:0] = [REPO, os.path.join(REPO, "sparc-gym_amd")]
    import bench
    from oracle.cpu_ref import CpuRefEnv
    proc = bench.make_pool(1024, *bench.CONFIGS["c3r"][:2], workers=1)[:64]
    co = RulesCOracle(proc)
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    rng = np.random.default_rng(7)
    seen = set()
    for q in range(len(proc)):
        env = CpuRefEnv(pool[q], True, 2000)
        for _ in range(40):
            _, term, trunc = env.step(int(rng.integers(4)))
            want = rules_ref.rule_bits(rules_ref.audit(proc[q], env.path, env.loc))
            assert co.bits(q, env.path, env.loc) == want, (q, env.path)
            seen.add(want)
            if term or trunc:
                break
    assert len(seen) > 8   # many different rule outcomes
