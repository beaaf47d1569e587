"""CPU model of the W = 1 split kernel's hand-over word (sparc_move1.hpp) and of the I/O wave's
SWAR flag bytes (flag_bytes4, sparc_kernels.hip): every combination of at-target / done /
autoreset / fwd - pop and every legal window, four env-steps per dword as the I/O wave packs
them, against the flag byte the reference's step() reports (term | trunc << 1 | legal << 2 |
autoreset << 6).  The GPU parity tests check the same bytes end to end; this pins the bit logic
itself without a GPU."""
import itertools

import numpy as np
import pytest

K_TGT, K_DONE = 1 << 24, 1 << 25


def legal_magic(P):
    return (1 << (18 - 2 * P)) + (1 << (20 - P)) + (1 << 20)


def window_positions(P):   # right, up, left, down (legal bits 0..3)
    return [2 * P, P - 1, 0, P + 1]


def hand_word(lw, at_tgt, done, reset, dl):
    """MoveLane1::step_pos: lw | (at_tgt or reset) << 24 | (done and not reset) << 25 | dl << 30."""
    pending = done and not reset
    return ((dl & 3) << 30) | (K_TGT if (at_tgt or reset) else 0) | (K_DONE if pending else 0) | lw


def flag_bytes4(words, P):
    """flag_bytes4: four words -> four flag bytes, bit for bit as the device code."""
    m = [(w & 0xFFFFFF) * legal_magic(P) & 0xFFFFFFFF for w in words]   # v_mul_u32_u24 (low 32 bits)

    def bytes4(ws, b):
        return sum(((ws[j] >> (8 * b)) & 0xFF) << (8 * j) for j in range(4))

    L = bytes4(m, 2) & 0x3C3C3C3C
    B = bytes4(words, 3)
    term = B & (B >> 1) & 0x01010101
    trunc = B & ~(B << 1) & 0x02020202
    rs = (B << 6) & ~(B << 5) & 0x40404040
    return (term | trunc | L | rs) & 0xFFFFFFFF


def reference_flag(legal, at_tgt, done, reset):
    if reset:   # an autoreset step is never done; its legal set is the new start's
        return (legal << 2) | 64
    term = at_tgt and done
    trunc = done and not at_tgt
    return int(term) | (int(trunc) << 1) | (legal << 2)


@pytest.mark.parametrize("P", [3, 5, 8, 9])
def test_flag_bytes_match_the_reference_flag_byte(P):
    pos = window_positions(P)
    cases = []
    for legal in range(16):
        lw = sum(1 << pos[d] for d in range(4) if legal >> d & 1)
        for at_tgt, done, reset, dl in itertools.product([0, 1], [0, 1], [0, 1], [-1, 0, 1]):
            if at_tgt and not done and not reset:
                continue                  # at the target is always done
            if reset and (dl != 0 or at_tgt):
                continue                  # an autoreset step neither moves nor starts at the target
            cases.append((hand_word(lw, at_tgt, done, reset, dl), reference_flag(legal, at_tgt, done, reset)))
    rng = np.random.default_rng(P)
    order = rng.permutation(len(cases))
    for k in range(0, len(order) - 3, 4):
        ws = [cases[i][0] for i in order[k:k + 4]]
        want = sum(cases[i][1] << (8 * j) for j, i in enumerate(order[k:k + 4]))
        assert flag_bytes4(ws, P) == want


def test_trie_wave_reset_and_move_decoding():
    """TrieLane: hw_reset (byte 3 == 1), done (bit 25), moved (bit 30) and fwd - pop (bits 30-31,
    sign-extended) from the word."""
    for at_tgt, done, reset, dl in itertools.product([0, 1], [0, 1], [0, 1], [-1, 0, 1]):
        if (at_tgt and not done and not reset) or (reset and (dl != 0 or at_tgt)):
            continue
        w = hand_word(0x7FFFF, at_tgt, done, reset, dl)
        assert ((w >> 24) == 1) == bool(reset)
        assert bool(w & K_DONE) == bool(done and not reset)
        assert (w >= 0x40000000) == (dl != 0)
        sdl = np.int32(np.uint32(w)) >> 30
        assert int(sdl) == dl
