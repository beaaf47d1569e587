"""The rule audit on every pool the reference accepts (_validate_rules, SPaRC_Gym.py:714-853, has
no size limits), and the exact-fit queue past its first capacity.

* A pool with more than 65,536 poly/ylop instances and more than 32,768 distinct polyshapes
  (the rule table's instance / shape indices are 32 / 21 bits), with puzzles past the GPU
  search's list sizes: one with 17+ ylops (stacked monomino ylops reach cell counts below the GPU
  counters' -32) and one with 17+ distinct poly shapes.  Those puzzles' searches run on the host
  (sparc_rules_finish, exact_fit with 64-entry lists and 8 counter planes).  Rule bits of sampled
  envs after random rollouts equal the oracle (oracle/rules_ref.py); SPaRC_Gym(rule_status=True)
  constructs on the pool and its rule_status matches the oracle.  (A puzzle holds at most one
  instance per cell centre, 49 on a 15 x 15 lattice, so the GPU search's 64-poly list never
  overflows.)
* The exact-fit queue (65,536 entries at first) overflowing: with the GPU's node cap at 1 every
  search is queued; a generic rule rollout of 8,192 envs x 48 steps (393,216 audits) and a
  k_rules audit of 65,536 envs queue more than the queue holds, sparc_rules_finish grows it and
  runs the call again from the state it started from; bits, rewards, flags, stats and state equal
  the same calls with the default cap (no searches queued) and, on samples, the oracle.
"""
import numpy as np
import pytest

from oracle import rules_ref

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _state_points(vis_words, pitch, X, Y):
    pts = []
    for x in range(X):
        for y in range(Y):
            b = x * pitch + y
            if (int(vis_words[b >> 6]) >> (b & 63)) & 1:
                pts.append([x, y])
    return pts


def _oracle_bits(refp, st, i, pitch):
    p = refp[int(st["puzzle"][i])]
    path = _state_points(st["visited"][:, i], pitch, p["x_size"], p["y_size"])
    return rules_ref.rule_bits(rules_ref.audit(p, path, (int(st["x"][i]), int(st["y"][i]))))


def _add_instances(rec, rng, n_ylops, n_polys, shape_fn, up_to=False):
    """Add poly / ylop instances (shape_fn(k) -> 0/1 array) on free cell centres of a record
    (up_to: as many polys as there are free cells, at most n_polys)."""
    from sparc_gym_amd.puzzles import safe_load
    from sparc_gym_amd.synthetic import _dump
    text = safe_load(rec["text_visualization"])
    poly = safe_load(rec["polyshapes"]) or {}
    X, Y = 2 * rec["grid_size"]["width"] + 1, 2 * rec["grid_size"]["height"] + 1
    used = {(c["position"]["x"], c["position"]["y"]) for c in text["puzzle"]["cells"]
            if "type" in c["properties"]}
    free = [(x, y) for x in range(1, X, 2) for y in range(1, Y, 2) if (x, y) not in used]
    rng.shuffle(free)
    if up_to:
        n_polys = min(n_polys, len(free) - n_ylops)
    kinds = ["ylop"] * n_ylops + ["poly"] * n_polys
    assert len(free) >= len(kinds), (len(free), len(kinds))
    sid = 900000 + int(rng.integers(1000)) * 100
    for k, (kind, (x, y)) in enumerate(zip(kinds, free)):
        poly[str(sid + k)] = shape_fn(k)
        text["puzzle"]["cells"].append({"position": {"x": int(x), "y": int(y)},
                                        "properties": {"type": kind, "color": "red", "polyshape": sid + k}})
    rec = dict(rec)
    rec["text_visualization"] = _dump(text)
    rec["polyshapes"] = _dump(poly)
    return rec


def _walled(rec, shape_fn, n_ylops, n_polys):
    """A 15 x 15 record split by a wall of gap points at lattice column wx (SPaRC_Gym.py:423-454:
    gaps block the region flood): region 0, the cells left of the wall, holds one vertical
    7-cell bar poly per cell column (its exact fit succeeds); region 1 holds n_ylops / n_polys
    more instances (shape_fn(k)) whose area check fails.  With 17 ylops or 17 distinct poly
    shapes the puzzle is past the GPU search's lists, so region 0's search runs on the host."""
    from sparc_gym_amd.puzzles import safe_load
    from sparc_gym_amd.synthetic import _dump
    text = safe_load(rec["text_visualization"])
    sx, ex = text["puzzle"]["start"]["x"], text["puzzle"]["end"]["x"]
    wx = next(x for x in (4, 6, 8, 10, 2, 12) if x not in (sx, ex))
    cells = [c for c in text["puzzle"]["cells"] if (c["position"]["x"], c["position"]["y"]) != (wx, 0)]
    for y in range(15):
        cells.append({"position": {"x": wx, "y": y}, "properties": {"gap": True}})
    poly, sid = {}, 700000
    left = [(x, 1) for x in range(1, wx, 2)]
    right = [(x, y) for x in range(wx + 1, 15, 2) for y in range(1, 15, 2)]
    poly[str(sid)] = [[1] * 7]   # dx = array row, dy = array column (_get_offsets 840-855)
    inst = [(c, "poly", sid) for c in left]
    for k in range(n_ylops + n_polys):
        poly[str(sid + 1 + k)] = shape_fn(k)
        inst.append((right[k], "ylop" if k < n_ylops else "poly", sid + 1 + k))
    for (x, y), kind, i in inst:
        cells.insert(0, {"position": {"x": x, "y": y}, "properties": {"type": kind, "color": "red", "polyshape": i}})
    text["puzzle"]["cells"] = cells
    rec = dict(rec)
    rec["text_visualization"] = _dump(text)
    rec["polyshapes"] = _dump(poly)
    return rec


def _two_walls(rec):
    """A 15 x 15 record with gap walls at lattice columns 2 and 12 and a vertical 7-cell bar poly
    in each outer cell column (x = 1, 13), or None when the start is not between the walls: the
    agent can never enter the outer regions, so every audit of this puzzle runs two exact-fit
    searches (both fit)."""
    from sparc_gym_amd.puzzles import safe_load
    from sparc_gym_amd.synthetic import _dump
    text = safe_load(rec["text_visualization"])
    if not 4 <= text["puzzle"]["start"]["x"] <= 10:
        return None
    cells = [c for c in text["puzzle"]["cells"] if c["position"]["x"] not in (2, 12)]
    cells += [{"position": {"x": x, "y": y}, "properties": {"gap": True}} for x in (2, 12) for y in range(15)]
    cells = [{"position": {"x": x, "y": 1}, "properties": {"type": "poly", "color": "red", "polyshape": 700000}}
             for x in (1, 13)] + cells
    text["puzzle"]["cells"] = cells
    rec = dict(rec)
    rec["text_visualization"] = _dump(text)
    rec["polyshapes"] = _dump({"700000": [[1] * 7]})
    return rec


def _limits_pool(n_base=1700):
    """n_base 15 x 15 puzzles (synthetic, base planes) with 40 polys each of random 5 x 5 shapes (more than 65,536 instances and 32,768 distinct shapes in all), then two puzzles past
    the GPU search's lists on an empty 15 x 15 base: 17 monomino ylops + 20 monomino polys (every
    region whose area check passes fits, and cell counts reach -18), and 17 polys of distinct
    shapes whose area fails every region (the flag and the loader, no search)."""
    from sparc_gym_amd import synthetic
    rng = np.random.default_rng(77)

    def random_shape(_k):   # 5 x 5, first cell set
        s = (rng.random((5, 5)) < 0.5).astype(int)
        s[0, 0] = 1
        return s.tolist()

    recs = [_add_instances(r, rng, 0, 40, random_shape, up_to=True)
            for r in synthetic.make_puzzles(n_base, seed=31, sizes=((7, 7),), full_properties=False, n_solutions=1)]
    empty = synthetic.make_puzzles(2, seed=32, sizes=((7, 7),), full_properties=False)
    rects = [(4, 5), (5, 4), (4, 6), (6, 4), (5, 5), (4, 7), (7, 4), (5, 6), (6, 5), (5, 7), (7, 5), (6, 6),
             (6, 7), (7, 6), (7, 7), (3, 7), (7, 3)]
    recs.append(_walled(empty[0], lambda k: [[1]], 17, 0))
    recs.append(_walled(empty[1], lambda k: [[1] * rects[k][1]] * rects[k][0], 0, 17))
    return recs


@pytest.fixture(scope="module")
def limits_pool():
    from sparc_gym_amd.puzzles import pack_rules, pack_table, process_puzzles
    recs = _limits_pool()
    proc = process_puzzles(recs)
    table = pack_table(proc)
    rt = pack_rules(proc, table)
    return recs, proc, table, rt


def test_rule_table_without_pool_limits_vs_oracle(on_gpu, limits_pool):
    from sparc_gym_amd import SPaRCVecEnv
    recs, proc, table, rt = limits_pool
    assert len(rt.inst) > 65536 and len(rt.shape_area) > 32768
    counts = []
    for q in range(len(proc)):
        f, c = rt.inst_range(q)
        e = rt.inst[f:f + c]
        ny = int(((e >> 10) & 1).sum())
        nd = len({int(s) for s in (e >> 11)[((e >> 10) & 1) == 0]})
        counts.append((ny, nd))
    flagged = [q for q, (ny, nd) in enumerate(counts) if ny > 16 or nd > 16]
    assert any(counts[q][0] > 16 for q in flagged) and any(counts[q][1] > 16 for q in flagged)
    n = 4096
    rng = np.random.default_rng(4)
    # half of the envs on the flagged puzzles, the rest over the pool
    pids = np.where(np.arange(n) % 2 == 0, np.array(flagged)[np.arange(n) % len(flagged)],
                    rng.integers(len(proc), size=n))
    vec = SPaRCVecEnv(n, processed=proc, table=table, traceback=True, autoreset="next_step",
                      observation="compact", rules=True, max_steps=60)
    vec.reset(options={"puzzle_index": pids})
    # the resets' audits queue the walled puzzles' region 0 (host-only fits): the host runs them
    searches = vec.core.rules_queue_stats()["last_searches"]
    refp = [dict(p) for p in proc]
    walled = [len(proc) - 2, len(proc) - 1]
    assert counts[walled[0]][0] == 17 and counts[walled[1]][1] >= 17
    pids[:64] = walled[0]
    pids[64:128] = walled[1]
    vec.reset(options={"puzzle_index": pids})
    searches += vec.core.rules_queue_stats()["last_searches"]
    assert searches >= 64
    for T in (0, 3, 9, 17):
        if T:
            vec.rollout(T, None, seed=T, record=False)
        out = vec.rule_audit(fit=True)
        bits = out["bits"].cpu().numpy().astype(np.uint16)
        assert not (bits & (1 << 9)).any()
        st = vec.state()
        sample = np.concatenate([np.arange(0, n, 2)[rng.choice(n // 2, 150, replace=False)],
                                 rng.choice(n, 100, replace=False)])
        for i in sample:
            assert int(bits[i]) == _oracle_bits(refp, st, i, table.pitch), (T, i, int(st["puzzle"][i]))
        if T == 0:   # region 0 of the walled puzzles fits: the host's answers, kept from the resets
            fit = out["fit"].cpu().numpy()
            assert ((fit[:128] & 1) == 1).all()
            assert vec.core.rules_queue_stats()["last_searches"] == 0


def test_sparc_gym_constructs_on_the_limits_pool(on_gpu, limits_pool):
    """SPaRC_Gym(rule_status=True) packs the rule table in its constructor (as the reference
    audits at load, SPaRC_Gym.py:182): it constructs on this pool, and its rule_status after
    steps on the flagged puzzles equals the oracle's."""
    from sparc_gym_amd import SPaRC_Gym
    recs, proc, table, rt = limits_pool
    env = SPaRC_Gym(puzzles=recs, traceback=True, rule_status=True)
    rng = np.random.default_rng(9)
    checked = 0
    for q in (len(recs) - 2, len(recs) - 1):   # the 17-ylop puzzle, the 17-distinct-shape puzzle
        env.reset(options={"puzzle_id": recs[q]["id"]})                               # SPaRC_Gym.py:1073-1079
        assert env.current_puzzle_index == q
        p = dict(env.puzzles[q])
        for _ in range(12):
            _, _, term, trunc, info = env.step(int(rng.integers(4)))
            want = rules_ref.normalize(rules_ref.audit(p, [list(v) for v in env.path], tuple(info["agent_location"])))
            got = rules_ref.normalize(info["rule_status"])
            for k in want:
                if k not in ("_terminated", "_truncated"):
                    assert got[k] == want[k], (q, k)
            checked += 1
            if term or trunc:
                break
    assert checked >= 2


@pytest.mark.parametrize("generic", [True, False])
def test_exact_fit_queue_overflow_rerun(on_gpu, generic):
    """fit_cap = 1: every exact-fit search is queued.  On a pool of two-walled puzzles
    (_two_walls: two searches per audit, none on the GPU; 15 x 15 lattices have no region-code
    table, so rule rollouts take the generic rule kernel) a rule rollout of 8,192 envs x 48 steps
    (393,216 audits) queues far more searches than the first queue holds, and so does one k_rules
    audit of 65,536 envs.  Their outputs equal the default cap's (every search on the GPU).  The
    host's answers are not kept here (SPARC_VARIANT_HOST_FITS = 1): kept, the reset's audit would
    answer every later search of this pool (test_host_fit_answers_are_kept)."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = [r for r in map(_two_walls, synthetic.make_puzzles(200, seed=41, sizes=((7, 7),), full_properties=False,
                                                                n_solutions=1)) if r is not None]
    assert len(recs) > 50
    proc = process_puzzles(recs)
    refp = [dict(p) for p in proc]
    if generic:
        n, T = 8192, 48
        pids = np.arange(n) % len(proc)
        acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda")
        runs = []
        for cap in (1, None):
            v = SPaRCVecEnv(n, processed=proc, traceback=True, autoreset="next_step", observation="compact",
                            rules=True, max_steps=40, fit_cap=cap)
            v.core.set_variant(v.core.VARIANT_HOST_FITS, 1)
            v.reset(options={"puzzle_index": pids})
            st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
            r = v.rollout(T, acts, rules=True, stats=st)
            runs.append(([r[k].cpu().numpy() for k in ("reward_code", "flags", "rule_bits")], st.cpu().numpy(),
                         v.state(), v))
        (a, sa, xa, va), (b, sb, xb, _) = runs
        for u, w in zip(a, b):
            assert np.array_equal(u, w)
        assert np.array_equal(sa, sb)
        for k in ("x", "y", "step", "path_len", "puzzle", "outcome", "visited"):
            assert np.array_equal(xa[k], xb[k]), k
        assert va.core.rules_queue_stats()["capacity"] > 65536   # the queue grew: the call ran again
        bits = a[2].astype(np.uint16)
        rng = np.random.default_rng(1)
        for i in rng.choice(n, 60, replace=False):
            assert int(bits[T - 1, i]) == _oracle_bits(refp, xa, i, va.table.pitch)
    else:
        n = 65536
        pids = np.arange(n) % len(proc)
        outs = []
        for cap in (1, None):
            v = SPaRCVecEnv(n, processed=proc, traceback=True, autoreset="next_step", observation="compact",
                            rules=True, max_steps=40, fit_cap=cap)
            v.core.set_variant(v.core.VARIANT_HOST_FITS, 1)
            v.reset(options={"puzzle_index": pids})
            v.rollout(7, None, seed=3, record=False)
            o = v.rule_audit(region=True, fit=True)
            outs.append(({k: o[k].cpu().numpy() for k in ("bits", "region", "fit")}, v))
        (a, va), (b, _) = outs
        for k in ("bits", "region", "fit"):
            assert np.array_equal(a[k], b[k]), k
        assert va.core.rules_queue_stats()["capacity"] > 65536
