"""Python model of the device rule audit (csrc/sparc_rules.hpp), on the packed RulesTable.

Mirrors the kernel's formulation (multi-word bitboards as Python ints, flood fill, bit-plane
popcounts, bit-sliced triangle counts, the iterative exact-fit search with its pruning) so the
CPU suite can check that formulation and `pack_rules` against the oracle before any GPU run.
"""
from sparc_gym_amd.puzzles import (RP_CELLS, RP_COL1, RP_COLORED, RP_DOTS, RP_GAPS, RP_LATTICE, RP_M0,
                                   RP_NOTFIRST, RP_NOTLAST, RP_SQUARE, RP_STAR, RP_TRI, RP_TRI0)

FIT_CAP = 1 << 26


def _bb(words):
    return sum(int(w) << (64 * k) for k, w in enumerate(words))


def exact_fit(rt, first, count, Rc, pitch, CX, CY):
    NC = CX * CY
    g = [(-1 if (Rc >> ((2 * (k // CY) + 1) * pitch + 2 * (k % CY) + 1)) & 1 else 0) for k in range(NC)]
    ysh, dsh, cnt = [], [], []
    for k in range(count):
        e = int(rt.inst[first + k])
        if not (Rc >> (e & 0x3FF)) & 1:
            continue
        sh = e >> 11
        if (e >> 10) & 1:
            ysh.append(sh)
        elif sh in dsh:
            cnt[dsh.index(sh)] += 1
        else:
            dsh.append(sh)
            cnt.append(1)
    ysh.sort()
    ny, npoly = len(ysh), sum(cnt)

    def offs(sh):
        return rt.shape_offsets(sh)

    def place(sh, a, sign):
        ax, ay = divmod(a, CY)
        t = [(ax + dx, ay + dy) for dx, dy in offs(sh)]
        if any(not (0 <= tx < CX and 0 <= ty < CY) for tx, ty in t):
            return False
        for tx, ty in t:
            g[tx * CY + ty] += sign
        return True

    def unplace(sh, a, sign):
        ax, ay = divmod(a, CY)
        for dx, dy in offs(sh):
            g[(ax + dx) * CY + ay + dy] -= sign

    cur = [-1] * (ny + npoly + 1)
    pat = [0] * (npoly + 1)
    L, it = 0, 0
    while True:
        it += 1
        assert it <= FIT_CAP
        if L < ny:
            a = cur[L]
            if a >= 0:
                unplace(ysh[L], a, -1)
            a = ((cur[L - 1] if L > 0 and ysh[L] == ysh[L - 1] else 0) if a < 0 else a + 1)
            while a < NC and not place(ysh[L], a, -1):
                a += 1
            if a >= NC:
                cur[L] = -1
                if L == 0:
                    return False
                L -= 1
                continue
            cur[L] = a
            L += 1
            cur[L] = -1
            continue
        lv = L - ny
        j = cur[L]
        if j < 0:
            pos = any(v > 0 for v in g)
            t = next((k for k, v in enumerate(g) if v < 0), -1)
            if pos or L == ny + npoly or t < 0:
                ok = (not pos) and (t < 0)
                if ok:
                    return True
                if L == 0:
                    return False
                L -= 1
                continue
            pat[lv] = t
        else:
            unplace(dsh[j], pat[lv], +1)
            cnt[j] += 1
        j += 1
        while j < len(dsh) and (cnt[j] == 0 or not place(dsh[j], pat[lv], +1)):
            j += 1
        if j >= len(dsh):
            cur[L] = -1
            if L == 0:
                return False
            L -= 1
            continue
        cnt[j] -= 1
        cur[L] = j
        L += 1
        cur[L] = -1


def audit(rt, table, q, vis, x, y):
    """(bits, fit_ok, {bit: region id}) for env state (vis bitboard int, agent x, y) on puzzle q."""
    W, P = table.words, table.pitch
    pl = [_bb(rt.planes[q, k]) for k in range(rt.planes.shape[1])]
    info = table.info[q]
    X, Y = int(info[0]) & 0xFF, (int(info[0]) >> 8) & 0xFF
    tx, ty = int(info[1]) & 0xFF, (int(info[1]) >> 8) & 0xFF
    full = (1 << (64 * W)) - 1
    cells, lattice, gaps = pl[RP_CELLS], pl[RP_LATTICE], pl[RP_GAPS]
    allowed = (lattice & ~(gaps | vis) | cells) & full
    first, count = rt.inst_range(q)
    sq_ok = star_ok = poly_ok = True
    fit_ok, rid, rmap = 0, 0, {}
    remaining = cells
    while remaining:
        R = remaining & -remaining
        while True:
            N = (R | ((R << 1) & pl[RP_NOTFIRST]) | ((R >> 1) & pl[RP_NOTLAST]) | (R << P) | (R >> P)) & allowed
            if N == R:
                break
            R = N
        Rc = R & cells
        remaining &= ~Rc
        for b in range(64 * W):
            if (Rc >> b) & 1:
                rmap[b] = rid
        sq = Rc & pl[RP_SQUARE]
        if sq:
            sq_ok &= sum(1 for c in range(8) if sq & pl[RP_COL1 + c]) <= 1
        st = Rc & pl[RP_STAR]
        if st:
            star_ok &= not (st & ~pl[RP_COLORED])
            for c in range(8):
                col = Rc & pl[RP_COL1 + c]
                if st & col:
                    tot = sum((1 << k) * bin(col & pl[RP_M0 + k]).count("1") for k in range(3))
                    star_ok &= tot == 2
        pa = ya = 0
        has = False
        for k in range(count):
            e = int(rt.inst[first + k])
            if (Rc >> (e & 0x3FF)) & 1:
                has = True
                a = int(rt.shape_area[e >> 11])
                if (e >> 10) & 1:
                    ya += a
                else:
                    pa += a
        if has:
            ok = bin(Rc).count("1") == pa - ya
            if ok:
                ok = exact_fit(rt, first, count, Rc, P, (X - 1) // 2, (Y - 1) // 2)
            if ok:
                fit_ok |= 1 << (rid & 63)
            poly_ok &= ok
        rid += 1
    a, b, c, d = vis >> P, (vis << P) & full, vis >> 1, (vis << 1) & full
    s1, c1, s2, c2 = a ^ b, a & b, c ^ d, c & d
    n0, k0 = s1 ^ s2, s1 & s2
    n1, n2 = c1 ^ c2 ^ k0, c1 & c2
    bad = pl[RP_TRI] & ((n0 ^ pl[RP_TRI0]) | (n1 ^ pl[RP_TRI0 + 1]) | (n2 ^ pl[RP_TRI0 + 2]))
    bits = (int(x == tx and y == ty) | 2 | (int(not (gaps & vis)) << 2) | (int(not (pl[RP_DOTS] & ~vis)) << 3)
            | (int(sq_ok) << 4) | (int(star_ok) << 5) | (int(not bad) << 6) | (int(poly_ok) << 7))
    bits |= int((bits & 0xFF) == 0xFF) << 8
    return bits, fit_ok, rmap
