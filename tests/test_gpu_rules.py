"""GPU parity of the rule audit (k_rules through the C ABI): the pass bits, region map and
exact-fit results against the reference's rule_status golden vectors, SPaRC_Gym's full
info['rule_status'] dict against the same vectors, and the bits at the benchmark's 65,536 envs
against the oracle (oracle/rules_ref.py) on a sample of envs."""
import numpy as np
import pytest

from golden_io import load
from oracle import rules_ref
from rules_io import RULE_POOLS, ref_puzzle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _fit_mask(status):
    m = 0
    for d in status["poly_ylop_area"]["detail"].get("region_details", []):
        if d["ok"]:
            m |= 1 << int(d["region"])
    return m


def _region_bits(refp, s, pitch, words):
    _, rm = rules_ref.RuleAudit(refp, s["path"], s["agent"]).compute_regions()
    out = np.full(64 * words, 255, np.uint8)
    for x in range(rm.shape[0]):
        for y in range(rm.shape[1]):
            if rm[x, y] >= 0:
                out[x * pitch + y] = rm[x, y]
    return out


# fit_cap 1: nearly every exact-fit search passes the GPU's node cap and is finished on the host
# (sparc_rules_finish for the audits, sparc_load_rules for the region-code table), so the answers
# of the reference's unbounded search (SPaRC_Gym.py:738-853) must come from that fallback
@pytest.mark.parametrize("fit_cap", [None, 1])
@pytest.mark.parametrize("pool", RULE_POOLS)
def test_vec_rules_match_reference(on_gpu, pool, fit_cap):
    from sparc_gym_amd import SPaRCVecEnv
    g = load(pool)
    eps = g["episodes"]
    n, T = len(eps), max(len(e["actions"]) for e in eps)
    vec = SPaRCVecEnv(n, puzzles=g["records"], traceback=g["traceback"], max_steps=2000, autoreset="none",
                      rules=True, fit_cap=fit_cap)
    refp = [ref_puzzle(p) for p in g["processed"]]
    pitch, words = vec.table.pitch, vec.table.words
    _, info = vec.reset(options={"puzzle_index": [e["puzzle_index"] for e in eps]})
    acts = np.full((T, n), 255, np.int64)
    for i, e in enumerate(eps):
        acts[:len(e["actions"]), i] = e["actions"]
    for t in range(-1, T):
        if t >= 0:
            vec.step(torch.from_numpy(acts[t]).cuda())
        r = vec.rule_audit(region=True, fit=True)
        bits = r["bits"].cpu().numpy().astype(np.uint16)
        region, fit = r["region"].cpu().numpy(), r["fit"].cpu().numpy().astype(np.uint64)
        for i, e in enumerate(eps):
            if t >= len(e["steps"]):
                continue
            s = e["reset"] if t < 0 else e["steps"][t]
            assert int(bits[i]) == rules_ref.rule_bits(s["rule_status"]), (pool, i, t)
            assert int(fit[i]) == _fit_mask(s["rule_status"]), (pool, i, t)
            assert np.array_equal(region[i], _region_bits(refp[e["puzzle_index"]], s, pitch, words)), (pool, i, t)


@pytest.mark.parametrize("fit_cap", [None, 1])
@pytest.mark.parametrize("pool", RULE_POOLS)
def test_single_env_rule_status_matches_reference(on_gpu, pool, fit_cap):
    """SPaRC_Gym's info['rule_status'] equals the reference's, the whole nested dict (with the GPU's
    exact-fit node cap at 1, through the host fallback: never an unknown answer)."""
    from sparc_gym_amd import SPaRC_Gym
    g = load(pool)
    env = SPaRC_Gym(puzzles=g["records"], traceback=g["traceback"], max_steps=2000, fit_cap=fit_cap)
    ids = [r["id"] for r in g["records"]]
    for e, ep in enumerate(g["episodes"][:12]):
        _, info = env.reset(options={"puzzle_id": ids[ep["puzzle_index"]]})
        assert rules_ref.normalize(info["rule_status"]) == ep["reset"]["rule_status"], (pool, e)
        for t, (a, s) in enumerate(zip(ep["actions"], ep["steps"])):
            _, _, _, _, info = env.step(a)
            assert rules_ref.normalize(info["rule_status"]) == s["rule_status"], (pool, e, t)
            assert info["rule_status"] is env.rule_status


def _state_points(vis_words, pitch, X, Y):
    v = sum(int(w) << (64 * k) for k, w in enumerate(vis_words))
    return [[x, y] for x in range(X) for y in range(Y) if (v >> (x * pitch + y)) & 1]


# unbounded random symbol soups only up to 11x11: on 13x13 / 15x15 boards they can hold regions
# with many ylops, whose exact-fit search (anchors^ylops, as in the reference) is effectively
# unbounded; there the soup is capped at 4 poly / ylop cells per puzzle (max_shaped)
@pytest.mark.parametrize("sizes,full,n,max_shaped", [(((3, 3),), True, 65536, None),
                                                     (((2, 2), (3, 3), (4, 4), (5, 5)), True, 8192, None),
                                                     (((7, 7), (6, 6)), False, 4096, None),
                                                     (((7, 7), (6, 6)), True, 4096, 4)])
def test_rules_at_scale_vs_oracle(on_gpu, sizes, full, n, max_shaped):
    """After a device rollout of random actions, k_rules bits equal the oracle's on a sample."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = synthetic.make_rule_puzzles(256, seed=8, sizes=sizes, break_prob=0.3)
    if full:
        recs += synthetic.make_puzzles(256, seed=7, sizes=sizes, full_properties=True, max_shaped=max_shaped)
    proc = process_puzzles(recs)
    vec = SPaRCVecEnv(n, processed=proc, traceback=True, autoreset="next_step", observation="compact",
                      rules=True)
    gid = np.arange(n, dtype=np.uint64)
    vec.reset(options={"puzzle_index": (gid * 2654435761 % len(proc)).astype(np.int64)})
    refp = [dict(p) for p in proc]
    rng = np.random.default_rng(0)
    checked = 0
    for T in (0, 7, 40):
        if T:
            vec.rollout(T, None, seed=T, record=False)
        bits = vec.rule_audit()["bits"].cpu().numpy().astype(np.uint16)
        assert not (bits & (1 << 9)).any()   # no exact-fit search reached its node cap
        st = vec.state()
        for i in rng.choice(n, size=400, replace=False):
            q = int(st["puzzle"][i])
            p = refp[q]
            path = _state_points(st["visited"][:, i], vec.table.pitch, p["x_size"], p["y_size"])
            want = rules_ref.rule_bits(rules_ref.audit(p, path, (int(st["x"][i]), int(st["y"][i]))))
            assert int(bits[i]) == want, (T, i, q)
            checked += 1
    vec.core.sync()
    assert checked == 1200


@pytest.mark.parametrize("sizes,max_shaped", [(((3, 3),), None), (((2, 3), (3, 2), (2, 2), (1, 3)), None),
                                              (((2, 2), (3, 3), (4, 4), (5, 5)), None), (((7, 7), (6, 6)), 4)])
def test_rollout_rule_bits_every_step(on_gpu, sizes, max_shaped):
    """rollout(rules=True): the audit after every step inside the rollout launch (the reference
    audits every step(), SPaRC_Gym.py:1227) equals step()-by-step() rule_audit() bits, and the
    reward codes / flags equal a plain rollout's; the bits of a sample of envs and steps equal
    the oracle's audit (oracle/rules_ref.py) of the oracle state."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = synthetic.make_rule_puzzles(128, seed=3, sizes=sizes, break_prob=0.3)
    recs += synthetic.make_puzzles(128, seed=4, sizes=sizes, full_properties=True, max_shaped=max_shaped)
    proc = process_puzzles(recs)
    n, T = 1024, 24
    kw = dict(processed=proc, traceback=True, autoreset="next_step", observation="compact", rules=True,
              max_steps=10)
    pids = (np.arange(n) * 37) % len(proc)
    acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda")
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    ra = a.rollout(T, acts, rules=True)
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    rb = b.rollout(T, acts)
    assert torch.equal(ra["reward_code"], rb["reward_code"]) and torch.equal(ra["flags"], rb["flags"])
    c = SPaRCVecEnv(n, **kw)
    c.reset(options={"puzzle_index": pids})
    bits = ra["rule_bits"].cpu().numpy()
    refp = [dict(p) for p in proc]
    rng = np.random.default_rng(1)
    for t in range(T):
        _, _, _, _, info = c.step(acts[t])
        assert np.array_equal(bits[t], info["rule_bits"].cpu().numpy()), t
        if t % 6 == 5:   # and a sample against the oracle's audit of the same state
            st = c.state()
            for i in rng.choice(n, size=50, replace=False):
                p = refp[int(st["puzzle"][i])]
                path = _state_points(st["visited"][:, i], c.table.pitch, p["x_size"], p["y_size"])
                want = rules_ref.rule_bits(rules_ref.audit(p, path, (int(st["x"][i]), int(st["y"][i]))))
                assert int(bits[t, i]) & 0x1FF == want, (t, i)
    assert not (bits & (1 << 9)).any()   # no exact-fit search reached its node cap
    assert len(np.unique(bits)) > 4


@pytest.mark.parametrize("n", [200, 1000, 1040])
def test_rollout_rule_bits_ragged_batches(on_gpu, n):
    """Rule rollouts over batches that are not whole workgroups (k_rollout1r: the audit waves take
    a tile's env-steps in env-major order, so the jobs of missing envs and of a partial last tile
    are skipped inside a wave): 200 and 1000 envs (not multiples of 16: every step goes through the
    per-step path), 1040 (tiled, with a last group of 16 envs), an odd T split over two
    launches; the bits after every step equal step()-by-step() audits and the reward codes /
    flags / stats equal a plain rollout's."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = synthetic.make_rule_puzzles(96, seed=5, sizes=((3, 3),), break_prob=0.3)
    recs += synthetic.make_puzzles(96, seed=6, sizes=((3, 3),), full_properties=True)
    proc = process_puzzles(recs)
    T1, T2 = 21, 16
    kw = dict(processed=proc, traceback=True, autoreset="next_step", observation="compact", rules=True,
              max_steps=9)
    pids = (np.arange(n) * 29) % len(proc)
    acts = torch.randint(0, 5, (T1 + T2, n), dtype=torch.uint8, device="cuda")
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    sa = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    r1 = a.rollout(T1, acts[:T1], rules=True, stats=sa)
    r2 = a.rollout(T2, acts[T1:], rules=True, stats=sa)
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    sb = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    rb = b.rollout(T1 + T2, acts, stats=sb)
    assert torch.equal(torch.cat([r1["reward_code"], r2["reward_code"]]), rb["reward_code"])
    assert torch.equal(torch.cat([r1["flags"], r2["flags"]]), rb["flags"])
    assert torch.equal(sa, sb)
    bits = torch.cat([r1["rule_bits"], r2["rule_bits"]]).cpu().numpy()
    c = SPaRCVecEnv(n, **kw)
    c.reset(options={"puzzle_index": pids})
    for t in range(T1 + T2):
        _, _, _, _, info = c.step(acts[t])
        assert np.array_equal(bits[t], info["rule_bits"].cpu().numpy()), t
    assert len(np.unique(bits)) > 4


def test_rollout_rules_c3r_full_size(on_gpu):
    """The bench's c3r workload at the bench's launch shape (bench.py --config c3r): 65,536 envs of
    the c3 pool, traceback, next-step autoreset, uint8 actions in HBM, the audit after every step,
    TWO back-to-back 2,000-step launches through the bench's own C-ABI call
    (sparc_rollout_rules_device: k_rollout1r on this pool, 200 tiles of its rings per launch) with
    the state carried through HBM.  Reward codes, flags and stats equal the plain rollout's (the
    split kernel, itself oracle-pinned); the rule bits of 256 sampled envs at 200 steps spread over
    both launches (every step of the first and last tiles, the tile-ring wrap points RT - 1 / RT /
    2 RT - 1 of a sample of tiles, the steps either side of the launch boundary, and random steps)
    equal the oracle's audit (oracle/rules_ref.py) of the C oracle's state after that step
    (SPaRC_Gym.py:941-950, 1227)."""
    from oracle import COracle
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    proc = process_puzzles(synthetic.make_puzzles(1024, seed=0, sizes=((3, 3),), full_properties=True))
    n, T, L, RT = 65536, 2000, 2, 10
    pids = (np.arange(n, dtype=np.uint64) * 2654435761 % 1024).astype(np.int64)
    kw = dict(processed=proc, traceback=True, autoreset="next_step", observation="compact", rules=True,
              max_steps=2000)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    acts = torch.randint(0, 4, (L, T, n), dtype=torch.uint8, device="cuda", generator=g)
    a = SPaRCVecEnv(n, **kw)
    a.reset(options={"puzzle_index": pids})
    a._stream()
    sa = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    rew = torch.empty((L, T, n), dtype=torch.int8, device="cuda")
    flg = torch.empty((L, T, n), dtype=torch.uint8, device="cuda")
    bits = torch.empty((L, T, n), dtype=torch.int16, device="cuda")
    for k in range(L):   # bench.py run(): raw C-ABI calls on pre-validated buffers
        a.core.rollout_rules_device(T, acts[k].data_ptr(), rew[k].data_ptr(), flg[k].data_ptr(), sa.data_ptr(),
                                    bits[k].data_ptr())
    a.core.sync()
    b = SPaRCVecEnv(n, **kw)
    b.reset(options={"puzzle_index": pids})
    sb = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    for k in range(L):
        rb = b.rollout(T, acts[k], stats=sb)
        assert torch.equal(rew[k], rb["reward_code"]) and torch.equal(flg[k], rb["flags"]), k
    assert torch.equal(sa, sb)
    bits = bits.reshape(L * T, n).cpu().numpy().astype(np.uint16)
    assert not (bits & (1 << 9)).any()
    rng = np.random.default_rng(2)
    idx = np.sort(rng.choice(n, 256, replace=False))
    steps = set(range(RT)) | set(range(L * T - RT, L * T)) | {T - 2, T - 1, T, T + 1, T + RT - 1, T + RT}
    for tile in rng.choice(L * T // RT, 40, replace=False):
        steps |= {int(tile) * RT + RT - 1, int(tile) * RT + RT} - {L * T}
    steps |= set(int(x) for x in rng.choice(L * T, 120, replace=False))
    steps = sorted(steps)
    assert len(steps) >= 200 and min(steps) == 0 and max(steps) == L * T - 1
    pool = [{"x_size": p["x_size"], "y_size": p["y_size"], "start": list(p["start_location"]),
             "target": list(p["target_location"]), "solution_count": p["solution_count"],
             "solution_paths": p["solution_paths"], "gaps": p["obs_array"]["gaps"]} for p in proc]
    refp = [dict(p) for p in proc]
    o = COracle(pool, len(idx), True, 2000, autoreset=1)
    o.reset(pids[idx])
    an = acts.reshape(L * T, n)[:, torch.from_numpy(idx).cuda()].cpu().numpy()
    done = 0
    for t in steps:
        o.rollout(t + 1 - done, np.ascontiguousarray(an[done:t + 1]))
        done = t + 1
        st = o.state()
        for j, i in enumerate(idx):
            p = refp[int(st["pid"][j])]
            vis = st["visited"][j]
            path = [[x, y] for x in range(p["x_size"]) for y in range(p["y_size"]) if vis[x, y]]
            want = rules_ref.rule_bits(rules_ref.audit(p, path, (int(st["x"][j]), int(st["y"][j]))))
            assert int(bits[t, i]) == want, (t, i)
    assert len(np.unique(bits)) > 4


def test_rules_area_list_fallback_vs_oracle(on_gpu):
    """A pool holding a shape of area 144 (a 12 x 12 block: a cell's net instance area outside the
    loader's 8-bit area planes): sparc_load_rules then leaves the area check to the walk over each
    region's instance list (sparc_rules.hpp region_net_area); k_rules bits still equal the
    oracle's (_polyfit_check_area 700-709; the big shape fails every area check, as in the
    reference)."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    proc = process_puzzles(synthetic.make_rule_puzzles(256, seed=8, sizes=((3, 3),), break_prob=0.3))
    big = 0
    for p in proc:
        if isinstance(p["polyshapes"], dict) and p["polyshapes"] and big < 16:
            name = sorted(p["polyshapes"])[0]
            p["polyshapes"] = dict(p["polyshapes"])
            p["polyshapes"][name] = [[1] * 12 for _ in range(12)]
            big += 1
    assert big == 16
    n = 4096
    vec = SPaRCVecEnv(n, processed=proc, traceback=True, autoreset="next_step", observation="compact",
                      rules=True)
    vec.reset(options={"puzzle_index": np.arange(n) % len(proc)})
    refp = [dict(p) for p in proc]
    rng = np.random.default_rng(4)
    for T in (0, 9, 30):
        if T:
            vec.rollout(T, None, seed=T, record=False)
        bits = vec.rule_audit()["bits"].cpu().numpy().astype(np.uint16)
        st = vec.state()
        for i in rng.choice(n, size=300, replace=False):
            p = refp[int(st["puzzle"][i])]
            path = _state_points(st["visited"][:, i], vec.table.pitch, p["x_size"], p["y_size"])
            want = rules_ref.rule_bits(rules_ref.audit(p, path, (int(st["x"][i]), int(st["y"][i]))))
            assert int(bits[i]) == want, (T, i)
    vec.core.sync()


def _oracle_bits(refp, st, i, pitch):
    p = refp[int(st["puzzle"][i])]
    path = _state_points(st["visited"][:, i], pitch, p["x_size"], p["y_size"])
    return rules_ref.rule_bits(rules_ref.audit(p, path, (int(st["x"][i]), int(st["y"][i]))))


def test_exact_fit_fallback_queue_is_used_and_final(on_gpu):
    """With the GPU's node cap at 1 on a pool without region-code tables (13x13 / 15x15 lattices:
    the audit runs the memoised search itself), k_rules leaves searches pending
    (SPARC_RULE_SEARCH_EXHAUSTED) until sparc_rules_finish has run them on the host without a cap;
    afterwards no bit is pending and every sampled env equals the oracle's audit."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = synthetic.make_rule_puzzles(128, seed=11, sizes=((7, 7), (6, 6)), break_prob=0.3)
    recs += synthetic.make_puzzles(128, seed=12, sizes=((7, 7), (6, 6)), full_properties=True, max_shaped=4)
    proc = process_puzzles(recs)
    n = 2048
    vec = SPaRCVecEnv(n, processed=proc, traceback=True, autoreset="next_step", observation="compact", rules=True,
                      fit_cap=1)
    vec.reset(options={"puzzle_index": np.arange(n) % len(proc)})
    refp = [dict(p) for p in proc]
    rng = np.random.default_rng(5)
    pending_seen = 0
    for T in (0, 6, 25):
        if T:
            vec.rollout(T, None, seed=T, record=False)
        bits = torch.empty(n, dtype=torch.int16, device="cuda")
        vec.core.rules_device(bits.data_ptr())
        raw = bits.cpu().numpy().astype(np.uint16)
        pending_seen += int(((raw >> 9) & 1).sum())
        vec.core.rules_finish(bits.data_ptr())
        fin = bits.cpu().numpy().astype(np.uint16)
        assert not (fin & (1 << 9)).any()
        st = vec.state()
        for i in rng.choice(n, size=200, replace=False):
            assert int(fin[i]) == _oracle_bits(refp, st, i, vec.table.pitch), (T, i)
    assert pending_seen > 0   # the cap did stop searches on the GPU


@pytest.mark.parametrize("budget", [None, 40 * 512])
@pytest.mark.parametrize("generic", [False, True])
def test_rules_table_budget_cutoff_mixed_pool(on_gpu, generic, budget):
    """budget 40 * 512: a region-code table budget that covers only the first 40 puzzles of a 7x7
    pool (sparc_load_rules stops at kMaxRegEntries), so the later puzzles are audited by the
    memoised search and one pool mixes table and search puzzles (the rule rollout then takes the
    generic kernel k_rollout<1, ..., RULES>).  budget None: every puzzle in the table (k_rollout1r,
    or with the SPARC_VARIANT_RULE_ROLLOUT_GENERIC variant the generic kernel on the same pool).  With the node cap at 1
    as well, every step of a rule rollout equals step()-by-step() audits, and samples equal the
    oracle."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = synthetic.make_rule_puzzles(96, seed=21, sizes=((3, 3),), break_prob=0.3)
    recs += synthetic.make_puzzles(96, seed=22, sizes=((3, 3),), full_properties=True)
    proc = process_puzzles(recs)
    n, T = 1024, 20
    kw = dict(processed=proc, traceback=True, autoreset="next_step", observation="compact", rules=True,
              max_steps=12, rule_table_entries=budget, fit_cap=1)
    pids = (np.arange(n) * 7) % len(proc)
    acts = torch.randint(0, 4, (T, n), dtype=torch.uint8, device="cuda")
    a = SPaRCVecEnv(n, **kw)
    if generic:
        a.core.set_variant(a.core.VARIANT_RULE_ROLLOUT_GENERIC, 1)
    a.reset(options={"puzzle_index": pids})
    ra = a.rollout(T, acts, rules=True)
    bits = ra["rule_bits"].cpu().numpy().astype(np.uint16)
    assert not (bits & (1 << 9)).any()
    c = SPaRCVecEnv(n, **kw)
    c.reset(options={"puzzle_index": pids})
    refp = [dict(p) for p in proc]
    rng = np.random.default_rng(3)
    for t in range(T):
        _, _, _, _, info = c.step(acts[t])
        assert np.array_equal(bits[t], info["rule_bits"].cpu().numpy().astype(np.uint16)), t
        if t % 5 == 4:
            st = c.state()
            for i in rng.choice(n, size=60, replace=False):
                assert int(bits[t, i]) == _oracle_bits(refp, st, i, c.table.pitch), (t, i)
    assert len(np.unique(bits)) > 4


@pytest.mark.parametrize("shape", [1, 2, 3, 4, 5])
def test_rule_rollout_shapes_equal_default(on_gpu, shape):
    """Every compiled shape of the W = 1 rule rollout (sparc_set_variant SPARC_VARIANT_R1R_SHAPE: k_rollout1r <G, A, RT> =
    <4, 3, 12>, <2, 4, 12> and <2, 5, 10> (the round-6 default before 15-step tiles), and the
    incremental audits 3, 4 (RegionSet1: regions kept from step to step, re-flooded only where a
    step splits one) besides the default <2, 5, 15>) gives the same
    reward codes, flags, stats, rule bits and final state as the default shape (oracle-pinned by
    test_rollout_rules_c3r_full_size), over two launches (the second with a partial last tile) on
    a ragged batch (a partial last group)."""
    from sparc_gym_amd import SPaRCVecEnv, synthetic
    from sparc_gym_amd.puzzles import process_puzzles
    recs = synthetic.make_rule_puzzles(128, seed=31, sizes=((3, 3),), break_prob=0.3)
    recs += synthetic.make_puzzles(128, seed=32, sizes=((3, 3),), full_properties=True)
    proc = process_puzzles(recs)
    n, T1, T2 = 8192 + 96, 48, 29
    kw = dict(processed=proc, traceback=True, autoreset="next_step", observation="compact", rules=True,
              max_steps=40)
    pids = (np.arange(n) * 13) % len(proc)
    acts = torch.randint(0, 5, (T1 + T2, n), dtype=torch.uint8, device="cuda")

    def run(shape=0):
        v = SPaRCVecEnv(n, **kw)
        v.core.set_variant(v.core.VARIANT_R1R_SHAPE, shape)
        v.reset(options={"puzzle_index": pids})
        st = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
        r1 = v.rollout(T1, acts[:T1], rules=True, stats=st)
        r2 = v.rollout(T2, acts[T1:], rules=True, stats=st)
        s = v.state()
        return [torch.cat([r1[k], r2[k]]).cpu().numpy() for k in ("reward_code", "flags", "rule_bits")], st.cpu().numpy(), s

    want, wst, ws = run()
    got, gst, gs = run(shape)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    assert np.array_equal(gst, wst)
    for k in ("x", "y", "path_len", "step", "puzzle", "outcome", "pending", "visited"):
        assert np.array_equal(gs[k], ws[k]), k
    assert len(np.unique(want[2])) > 4
