"""The one-env round trip of the drop-in SPaRC_Gym (sparc_env_step / _reset / _read, VERDICT r5
item 2): the step, the new state and the rule audit come back in one pinned record after ONE
stream synchronisation.  The record equals what the separate calls return (sparc_step_host,
sparc_read_state, sparc_rules_host: their results are pinned to the reference by the golden
tests) on every step of random episodes, on 7 x 7, mixed 5 x 5 - 11 x 11 and 15 x 15 pools, with
and without traceback, and with the GPU's exact-fit node cap at 1 (every search finished on the
host inside the call).  Also the exact-fit answers the host finished are kept on the device
(ADVICE r5 medium): a second audit of the same states queues nothing.
"""
import numpy as np
import pytest

from sparc_gym_amd import synthetic
from sparc_gym_amd.puzzles import pack_rules, pack_table, process_puzzles

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

POOLS = {
    "7x7_full": dict(sizes=((3, 3),), full_properties=True),
    "mixed_5_11": dict(sizes=((2, 2), (3, 3), (4, 4), (5, 5), (2, 5), (5, 3)), full_properties=True),
    "15x15": dict(sizes=((7, 7), (6, 7)), full_properties=True),
}


def _cores(proc, tb, fit_cap):
    from sparc_gym_amd.core import SparcCore
    table = pack_table(proc)
    rt = pack_rules(proc, table)
    out = []
    for _ in range(2):
        c = SparcCore(table, 1, tb, 60, "none", 0)
        if fit_cap:
            c.set_rule_limits(fit_cap, 0)
        c.load_rules(rt)
        out.append(c)
    return table, out


def _check_record(rec, table, st, rules):
    W = table.words
    assert rec.x == st["x"][0] and rec.y == st["y"][0]
    assert rec.path_len == st["path_len"][0]
    assert rec.step == st["step"][0] and rec.puzzle == st["puzzle"][0]
    assert rec.outcome == st["outcome"][0] and rec.pending == st["pending"][0]
    assert list(rec.visited)[:W] == [int(v) for v in st["visited"][:, 0]]
    assert not any(rec.visited[W:])
    if rules is None:
        assert rec.audited == 0
        return
    assert rec.audited == 1
    assert rec.rule_bits == int(rules["bits"][0])
    assert not rec.rule_bits & (1 << 9)   # never a pending search
    assert rec.fit == int(rules["fit"][0])
    reg = np.frombuffer(rec.region, np.uint8)
    assert np.array_equal(reg[:64 * W], rules["region"][0])
    assert (reg[64 * W:] == 0xFF).all()


@pytest.mark.parametrize("name", list(POOLS))
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("fit_cap", [None, 1])
def test_env_record_equals_separate_calls(on_gpu, name, tb, fit_cap):
    proc = process_puzzles(synthetic.make_puzzles(24, seed=len(name) + 3 * tb, **POOLS[name]))
    table, (a, b) = _cores(proc, tb, fit_cap)
    rng = np.random.default_rng(5 + tb)
    host_fits = 0
    for episode in range(6):
        q = int(rng.integers(len(proc)))
        audit = episode != 3   # one episode without the audit
        rec = a.env_reset(q, audit=audit)
        flags = b.reset_host(np.array([q], np.uint32))
        assert rec.flags == flags[0] and rec.reward_code == 0
        _check_record(rec, table, b.read_state(), b.rules_host(region=True, fit=True) if audit else None)
        for t in range(70):
            act = int(rng.choice([0, 1, 2, 3, 0, 1, 2, 3, 4, -1]))
            rec = a.env_step(act, audit=audit)
            host_fits += rec.host_fits
            codes, fl = b.step_host(np.array([act if 0 <= act < 4 else 255], np.uint8))
            assert rec.reward_code == codes[0] and rec.flags == fl[0], (episode, t)
            _check_record(rec, table, b.read_state(), b.rules_host(region=True, fit=True) if audit else None)
            if fl[0] & 3 and t % 7 == 0:
                break
        # the read entry point: no transition
        rec2 = a.env_read(audit=True)
        _check_record(rec2, table, b.read_state(), b.rules_host(region=True, fit=True))
    # (whether the GPU's node cap queued searches depends on the episodes: the host-finish path
    # inside the call is pinned by test_env_record_host_finish below)


def test_env_record_host_finish(on_gpu):
    """With the GPU's node cap at 1, the audit of a two-walled puzzle (test_gpu_rules_limits
    _two_walls: two exact-fit searches per audit) queues both searches; sparc_env_reset /
    sparc_env_step finish them on the host inside the call (host_fits = 2, no pending bit) and
    the record equals the default cap's.  The host's answers are kept (HostFits): the next
    audit of the same regions queues nothing."""
    from test_gpu_rules_limits import _two_walls
    recs = [r for r in map(_two_walls, synthetic.make_puzzles(40, seed=41, sizes=((7, 7),), full_properties=False,
                                                               n_solutions=1)) if r is not None]
    proc = process_puzzles(recs)
    table, (a, _) = _cores(proc, True, 1)
    _, (b, _) = _cores(proc, True, None)
    ra = a.env_reset(0, audit=True)
    rb = b.env_reset(0, audit=True)
    assert ra.host_fits == 2 and rb.host_fits == 0
    for r in (ra, rb):
        assert r.audited == 1 and not r.rule_bits & (1 << 9)
    assert (ra.rule_bits, ra.fit, bytes(ra.region)) == (rb.rule_bits, rb.fit, bytes(rb.region))
    assert ra.fit & 1   # the left walled region (region 0) fits
    again = a.env_reset(0, audit=True)
    assert again.host_fits == 0 and (again.rule_bits, again.fit) == (ra.rule_bits, ra.fit)
    rng = np.random.default_rng(2)
    for _ in range(30):
        act = int(rng.integers(4))
        ra, rb = a.env_step(act, audit=True), b.env_step(act, audit=True)
        assert (ra.rule_bits, ra.fit, bytes(ra.region), ra.flags) == (rb.rule_bits, rb.fit, bytes(rb.region), rb.flags)
        assert not ra.rule_bits & (1 << 9)
        if ra.flags & 3:
            break


def test_env_record_errors(on_gpu):
    from sparc_gym_amd._lib import SparcError
    from sparc_gym_amd.core import SparcCore
    proc = process_puzzles(synthetic.make_puzzles(4, seed=1, **POOLS["7x7_full"]))
    table = pack_table(proc)
    c = SparcCore(table, 1, True, 60, "none", 0)
    with pytest.raises(SparcError):
        c.env_step(0)                       # no state yet
    c.env_reset(1)
    with pytest.raises(ValueError):
        c.env_reset(len(proc))              # puzzle index out of range
    with pytest.raises(ValueError):
        c.env_step(0, env=1)                # env index out of range
    with pytest.raises(SparcError):
        c.env_step(0, audit=True)           # no rule table
    rec = c.env_step(0)
    assert rec.step == 1 and rec.puzzle == 1


def test_sparc_gym_step_is_one_round_trip(on_gpu):
    """SPaRC_Gym.step / reset call sparc_env_step / sparc_env_reset exactly once and nothing else
    of the C ABI (one stream synchronisation per call, the audit included)."""
    from sparc_gym_amd import SPaRC_Gym
    recs = synthetic.make_puzzles(8, seed=3, **POOLS["7x7_full"])
    env = SPaRC_Gym(puzzles=recs, traceback=True, rule_status=True)
    calls = []
    lib = env._core.lib

    class Spy:
        def __getattr__(self, k):
            f = getattr(lib, k)

            def g(*args):
                calls.append(k)
                return f(*args)
            return g
    env._core.lib = Spy()
    env.reset(seed=3)
    assert calls == ["sparc_env_reset"], calls
    rng = np.random.default_rng(0)
    for _ in range(20):
        calls.clear()
        _, _, term, trunc, info = env.step(int(rng.integers(4)))
        assert calls == ["sparc_env_step"], calls
        assert "rule_status" in info and info["rule_status"]
        if term or trunc:
            break


def test_host_fit_answers_are_kept(on_gpu):
    """exact fits the host finished are kept on the device (HostFits), so an
    audit looks them up instead of queueing the same (puzzle, region) search again.  On the
    two-walled pool (two exact-fit searches per audit, 15 x 15: no region-code table) with the
    GPU's node cap at 1, the first audit (reset's) queues every search, later audits of the
    same regions and a rule rollout over the same puzzles queue none, and every result equals the default
    cap's (every search on the GPU)."""
    from sparc_gym_amd import SPaRCVecEnv
    from test_gpu_rules_limits import _two_walls
    recs = [r for r in map(_two_walls, synthetic.make_puzzles(60, seed=43, sizes=((7, 7),), full_properties=False,
                                                               n_solutions=1)) if r is not None]
    proc = process_puzzles(recs)
    n, T = 2048, 24
    pids = np.arange(n) % len(proc)
    outs = []
    for cap in (1, None):
        v = SPaRCVecEnv(n, processed=proc, traceback=True, autoreset="next_step", observation="compact",
                        rules=True, max_steps=40, fit_cap=cap)
        v.reset(options={"puzzle_index": pids})   # rules=True: reset() audits the fresh states
        first = v.core.rules_queue_stats()["last_searches"]
        v.rollout(5, None, seed=2, record=False)
        a1 = {k: x.cpu().numpy().copy() for k, x in v.rule_audit(region=True, fit=True).items()}
        second = v.core.rules_queue_stats()["last_searches"]
        a2 = {k: x.cpu().numpy().copy() for k, x in v.rule_audit(region=True, fit=True).items()}
        second += v.core.rules_queue_stats()["last_searches"]
        r = v.rollout(T, None, seed=4, rules=True)
        third = v.core.rules_queue_stats()["last_searches"]
        outs.append((a1, a2, r["rule_bits"].cpu().numpy(), r["reward_code"].cpu().numpy(), first, second, third))
    (a1, a2, rb, rc, first, second, third), (b1, b2, sb, sc, *_) = outs
    for k in a1:
        assert np.array_equal(a1[k], b1[k]) and np.array_equal(a2[k], b2[k]), k
    assert np.array_equal(rb, sb) and np.array_equal(rc, sc)
    assert first >= 2 * n and second == 0 and third == 0, (first, second, third)
