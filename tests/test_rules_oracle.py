"""The rule-audit oracle (oracle/rules_ref.py) against the reference's own rule_status, recorded
per step in tests/golden/rules_*.json.gz."""
import collections

import pytest

from golden_io import load
from oracle import rules_ref
from rules_io import RULE_POOLS, ref_puzzle, snapshots


@pytest.mark.parametrize("pool", RULE_POOLS)
def test_oracle_matches_reference_rule_status(pool):
    g = load(pool)
    puzzles = [ref_puzzle(p) for p in g["processed"]]
    n = 0
    for e, pi, t, s in snapshots(g):
        got = rules_ref.normalize(rules_ref.audit(puzzles[pi], s["path"], s["agent"]))
        assert got == s["rule_status"], (pool, e, t)
        n += 1
    assert n > 50


def test_golden_covers_every_rule_both_ways():
    seen = collections.Counter()
    for pool in RULE_POOLS:
        for *_, s in snapshots(load(pool)):
            for k in rules_ref.RULE_NAMES:
                seen[(k, s["rule_status"][k]["passed"])] += 1
            for d in s["rule_status"]["poly_ylop_area"]["detail"].get("region_details", []):
                seen[("exact_fit", d["exact_fit"]["ok"])] += 1
    for k in rules_ref.RULE_NAMES[2:] + ("exact_fit",):
        assert seen[(k, True)] > 0 and seen[(k, False)] > 0, k
