"""The device rule-audit formulation (tests/rules_model.py mirrors csrc/sparc_rules.hpp) and the
rule table packer, against the reference's rule_status (golden) and the oracle's region map."""
import pytest

from golden_io import load
from oracle import rules_ref
from rules_io import RULE_POOLS, ref_puzzle, snapshots
from rules_model import audit
from sparc_gym_amd.puzzles import pack_rules, pack_table, process_puzzles


def vis_bits(path, pitch):
    v = 0
    for x, y in path:
        v |= 1 << (x * pitch + y)
    return v


def fit_mask(status):
    m = 0
    for d in status["poly_ylop_area"]["detail"].get("region_details", []):
        if d["ok"]:
            m |= 1 << int(d["region"])
    return m


@pytest.mark.parametrize("pool", RULE_POOLS)
@pytest.mark.parametrize("words", [None, 2, 4])
def test_model_matches_reference(pool, words):
    g = load(pool)
    proc = process_puzzles(g["records"])
    try:
        table = pack_table(proc, words=words)
    except ValueError:
        pytest.skip(f"pool does not fit {words} words")
    rt = pack_rules(proc, table)
    refp = [ref_puzzle(p) for p in g["processed"]]
    for e, q, t, s in snapshots(g):
        bits, fit, rmap = audit(rt, table, q, vis_bits(s["path"], table.pitch), *s["agent"])
        assert bits == rules_ref.rule_bits(s["rule_status"]), (pool, e, t)
        assert fit == fit_mask(s["rule_status"]), (pool, e, t)
        _, region_map = rules_ref.RuleAudit(refp[q], s["path"], s["agent"]).compute_regions()
        want = {x * table.pitch + y: int(region_map[x, y])
                for x in range(region_map.shape[0]) for y in range(region_map.shape[1]) if region_map[x, y] >= 0}
        assert rmap == want, (pool, e, t)


def test_pack_rules_raises_like_the_reference_without_poly_layer():
    from sparc_gym_amd import synthetic
    import numpy as np
    import yaml
    r = synthetic.make_rule_puzzle(np.random.default_rng(1), 2, 2, break_prob=0.0)
    t = yaml.safe_load(r["text_visualization"])
    t["puzzle"]["cells"] = [{"position": {"x": 1, "y": 1}, "properties": {"type": "ylop", "color": "red", "polyshape": 5}}]
    r["text_visualization"] = yaml.safe_dump(t, sort_keys=False)
    r["polyshapes"] = yaml.safe_dump({"5": [[1]]})
    proc = process_puzzles([r])
    with pytest.raises(KeyError):
        pack_rules(proc, pack_table(proc))


@pytest.mark.parametrize("pool", RULE_POOLS)
def test_rule_status_layout_matches_reference(pool):
    """sparc_gym_amd.rules.rule_status (the dict layout SPaRC_Gym returns) fed with the modelled
    device outputs reproduces the reference's full rule_status."""
    import numpy as np
    from collections import OrderedDict
    from sparc_gym_amd.rules import region_map_of, rule_status
    g = load(pool)
    proc = process_puzzles(g["records"])
    table = pack_table(proc)
    rt = pack_rules(proc, table)
    for e, q, t, s in snapshots(g):
        p = proc[q]
        bits, fit, rmap = audit(rt, table, q, vis_bits(s["path"], table.pitch), *s["agent"])
        reg = np.full(64 * table.words, 255, np.uint8)
        for b, r in rmap.items():
            reg[b] = r
        obs = OrderedDict((k, v.copy()) for k, v in p["obs_array"].items())
        for x, y in s["path"]:
            obs["visited"][x, y] = 1
        got = rule_status(p, obs, s["path"], np.array(s["agent"]), np.array(p["target_location"]), bits,
                          region_map_of(reg, p["x_size"], p["y_size"], table.pitch), fit)
        assert rules_ref.normalize(got) == s["rule_status"], (pool, e, t)


def test_pending_exact_fit_bits_are_refused():
    """SPARC_RULE_SEARCH_EXHAUSTED marks an exact-fit search still pending on the host: the C ABI
    finishes every search past the GPU's node cap without a cap (sparc_rules_finish, which
    sparc_rules_host runs itself), so rule_status never sees the flag and never reports an
    unknown answer (no ``passed: None``); bits that still carry it are a caller error."""
    import numpy as np
    from collections import OrderedDict
    from sparc_gym_amd.rules import RULE_NAMES, RULE_SEARCH_EXHAUSTED, region_map_of, rule_status
    g = load("rules_7x7_tb1")
    proc = process_puzzles(g["records"])
    table = pack_table(proc)
    p = proc[0]
    obs = OrderedDict((k, v.copy()) for k, v in p["obs_array"].items())
    reg = np.full(64 * table.words, 255, np.uint8)
    args = (p, obs, [list(p["start_location"])], np.array(p["start_location"]), np.array(p["target_location"]))
    rmap = region_map_of(reg, p["x_size"], p["y_size"], table.pitch)
    other = sum(1 << k for k in range(9))
    with pytest.raises(RuntimeError, match="sparc_rules_finish"):
        rule_status(*args, RULE_SEARCH_EXHAUSTED | other, rmap, 0)
    rs = rule_status(*args, other, rmap, 0)
    assert all(rs[n]["passed"] is True for n in RULE_NAMES)
