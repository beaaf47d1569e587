/* sparc_rules_oracle.c — CPU restatement of the SPaRC-Gym rule audit, pass bits only.
 * TEST / BENCHMARK INFRASTRUCTURE ONLY: bench.py's c3r cpu_baseline leg (oracle/cpu_bench.py
 * --impl c_rules) and tests/test_rules_oracle_c.py load it; the product never does.
 *
 * A literal C port of oracle/rules_ref.py (itself pinned by tests/golden/rules_*.json.gz, made by
 * importing the reference), which follows /root/reference/SPaRC_Gym/SPaRC_Gym.py:
 *   _compute_regions 422-454 (the BFS over cell centres and free lattice points, with its quirk:
 *     a cell can be queued twice, so a region's cell list — and its area — can count it twice),
 *   _collect_region_symbols 456-481, _rule_reached_target 487-495, _rule_path_not_crossing
 *   497-505, _rule_no_gap_violations 507-517, _rule_all_dots_collected 519-531,
 *   _rule_square_color_separation 533-551, _rule_star_pairing_exact 553-619,
 *   _rule_triangles_edge_count 622-646, _rule_poly_ylop_area 648-709 with _polyfit_region_exact
 *   736-853 (ylops placed at every cell anchor, then polys at the first negative cell, distinct
 *   names only) and _validate_rules 896-950.
 * It shares no data structure with the GPU audit (bitboard floods, region-code tables).
 */
#include <stdint.h>
#include <string.h>

#include "sparc_oracle.h"

#define RD ORACLE_MAXDIM
#define RMAXSHAPE 32   /* cells per polyshape */

enum { L_OTHER = 0, L_STAR, L_SQUARE, L_TRIANGLE, L_POLY, L_DOT };

typedef struct {
    int32_t n_puzzles;
    const int32_t *dims;        /* [P][4]: x_size, y_size, target_x, target_y                      */
    const uint8_t *gaps;        /* [P][16][16]                                                     */
    const int32_t *color;       /* [P][16][16] color_array                                         */
    const int64_t *add;         /* [P][16][16] additional_info                                     */
    const int32_t *layer_first; /* [P] first symbol layer of puzzle p (obs_array keys past the skip set) */
    const int32_t *layer_count; /* [P]                                                             */
    const int32_t *layer_kind;  /* [Lt] L_* of each layer                                          */
    const uint8_t *layers;      /* [Lt][16][16]                                                    */
    const int32_t *shape_first; /* [P] polyshapes of puzzle p                                      */
    const int32_t *shape_count; /* [P]                                                             */
    const int64_t *shape_name;  /* [S] the name as an integer (str(additional_info value) == key)  */
    const int32_t *shape_ncell; /* [S] cells (its area)                                            */
    const int32_t *shape_off;   /* [S][RMAXSHAPE][2] _get_offsets (2 dx, 2 dy from the anchor)     */
} oracle_rules_pool;

typedef struct {
    int H, W, nreg;
    int32_t map[RD][RD];          /* region id of each cell centre, -1 elsewhere */
    int32_t area[RD * RD];        /* len(cells) per region (duplicates included) */
    uint8_t cell[RD * RD][RD][RD];/* the region's cell set (rmask of _polyfit_region_exact) */
} regions_t;

static void compute_regions(const oracle_rules_pool *rp, int q, const oracle_env *e, regions_t *R) {
    const int H = rp->dims[4 * q], W = rp->dims[4 * q + 1];
    const uint8_t *gaps = rp->gaps + (size_t)q * RD * RD;
    uint8_t mask2[RD][RD];
    for (int x = 0; x < H; ++x)
        for (int y = 0; y < W; ++y) mask2[x][y] = gaps[x * RD + y] == 1;
    for (int k = 0; k < e->path_len; ++k) mask2[e->path[k][0]][e->path[k][1]] = 1;
    R->H = H;
    R->W = W;
    R->nreg = 0;
    for (int x = 0; x < RD; ++x)
        for (int y = 0; y < RD; ++y) R->map[x][y] = -1;
    static const int D[4][2] = {{0, 1}, {0, -1}, {1, 0}, {-1, 0}};
    int qx[2 * RD * RD + 1], qy[2 * RD * RD + 1];
    for (int x = 0; x < H; ++x)
        for (int y = 0; y < W; ++y) {
            if (!((x & 1) && (y & 1)) || R->map[x][y] != -1) continue;
            const int rid = R->nreg++;
            uint8_t enq[RD][RD];
            memset(enq, 0, sizeof(enq));
            memset(R->cell[rid], 0, sizeof(R->cell[rid]));
            int head = 0, tail = 0;
            qx[tail] = x, qy[tail++] = y;
            R->map[x][y] = rid;
            int area = 0;
            while (head < tail) {
                const int cx = qx[head], cy = qy[head++];
                if ((cx & 1) && (cy & 1)) {
                    ++area;
                    R->cell[rid][cx][cy] = 1;
                }
                for (int d = 0; d < 4; ++d) {
                    const int nx = cx + D[d][0], ny = cy + D[d][1];
                    if (nx < 0 || nx >= H || ny < 0 || ny >= W) continue;
                    if ((nx & 1) && (ny & 1) && R->map[nx][ny] == -1) {
                        R->map[nx][ny] = rid;
                        qx[tail] = nx, qy[tail++] = ny;
                    }
                    if (!mask2[nx][ny] && !enq[nx][ny]) {
                        enq[nx][ny] = 1;
                        qx[tail] = nx, qy[tail++] = ny;
                    }
                }
            }
            R->area[rid] = area;
        }
}

/* exact fit (_polyfit_region_exact 736-853): grid[x][y] as there */
typedef struct { int n; const int32_t *off; int64_t name; } piece_t;

static int try_place(int g[RD][RD], int H, int W, const piece_t *p, int ax, int ay, int sign) {
    for (int k = 0; k < p->n; ++k) {
        const int tx = ax + p->off[2 * k], ty = ay + p->off[2 * k + 1];
        if (tx < 0 || tx >= H || ty < 0 || ty >= W) return 0;
    }
    for (int k = 0; k < p->n; ++k) g[ax + p->off[2 * k]][ay + p->off[2 * k + 1]] += sign;
    return 1;
}
static void unplace(int g[RD][RD], const piece_t *p, int ax, int ay, int sign) {
    for (int k = 0; k < p->n; ++k) g[ax + p->off[2 * k]][ay + p->off[2 * k + 1]] -= sign;
}

static int place_polys(int g[RD][RD], int H, int W, piece_t *polys, int np) {
    int anyneg = 0, nx = -1, ny = -1;
    for (int x = 0; x < H; ++x)
        for (int y = 0; y < W; ++y) {
            if (g[x][y] > 0) return 0;
            if (g[x][y] < 0 && !anyneg) anyneg = 1, nx = x, ny = y;   /* lexicographic first */
        }
    if (np == 0) return !anyneg;
    if (!anyneg) return 1;
    for (int i = 0; i < np; ++i) {
        int seen = 0;
        for (int j = 0; j < i; ++j) seen |= polys[j].name == polys[i].name;
        if (seen) continue;
        if (!try_place(g, H, W, &polys[i], nx, ny, +1)) continue;
        piece_t rest[64];
        int m = 0;
        for (int j = 0; j < np; ++j)
            if (j != i) rest[m++] = polys[j];
        if (place_polys(g, H, W, rest, m)) return 1;
        unplace(g, &polys[i], nx, ny, +1);
    }
    return 0;
}

static int place_ylops(int g[RD][RD], int H, int W, piece_t *ylops, int ny_, int idx, piece_t *polys, int np) {
    if (idx == ny_) return place_polys(g, H, W, polys, np);
    for (int ax = 1; ax < H; ax += 2)
        for (int ay = 1; ay < W; ay += 2) {
            if (!try_place(g, H, W, &ylops[idx], ax, ay, -1)) continue;
            if (place_ylops(g, H, W, ylops, ny_, idx + 1, polys, np)) return 1;
            unplace(g, &ylops[idx], ax, ay, -1);
        }
    return 0;
}

static int cmp_i64(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}
#include <stdlib.h>

static int polyfit_exact(const regions_t *R, int rid, piece_t *polys, int np, piece_t *ylops, int ny_) {
    int pa = 0, ya = 0;
    for (int i = 0; i < np; ++i) pa += polys[i].n;
    for (int i = 0; i < ny_; ++i) ya += ylops[i].n;
    const int net = pa - ya;
    if (net == 0 && np == ny_) {   /* Counter(poly names) == Counter(ylop names) */
        int64_t a[64], b[64];
        for (int i = 0; i < np; ++i) a[i] = polys[i].name, b[i] = ylops[i].name;
        qsort(a, np, sizeof(int64_t), cmp_i64);
        qsort(b, np, sizeof(int64_t), cmp_i64);
        if (!memcmp(a, b, sizeof(int64_t) * np)) return 1;
    }
    int g[RD][RD];
    memset(g, 0, sizeof(g));
    if (net > 0)
        for (int x = 0; x < R->H; ++x)
            for (int y = 0; y < R->W; ++y)
                if (R->cell[rid][x][y]) g[x][y] = -1;
    return place_ylops(g, R->H, R->W, ylops, ny_, 0, polys, np);
}

/* _validate_rules (896-950) pass bits, bit k = rules_ref.RULE_NAMES[k]; -1 on the reference's
 * KeyError (a poly / ylop instance in a puzzle without a 'poly' plane, 734) */
int oracle_rules_bits(const oracle_rules_pool *rp, int q, const oracle_env *e) {
    static regions_t R;   /* one audit at a time per process (the baseline is single-threaded) */
    compute_regions(rp, q, e, &R);
    const int H = R.H, W = R.W;
    const uint8_t *gaps = rp->gaps + (size_t)q * RD * RD;
    const int32_t *col = rp->color + (size_t)q * RD * RD;
    const int64_t *add = rp->add + (size_t)q * RD * RD;
    const int L0 = rp->layer_first[q], NL = rp->layer_count[q];
    /* reached_target 487-495 */
    const int reached = e->x == rp->dims[4 * q + 2] && e->y == rp->dims[4 * q + 3];
    /* path_not_crossing 497-505 */
    int crossing = 0;
    for (int i = 0; i < e->path_len && !crossing; ++i)
        for (int j = 0; j < i; ++j)
            if (e->path[i][0] == e->path[j][0] && e->path[i][1] == e->path[j][1]) { crossing = 1; break; }
    /* no_gap_violations 507-517 */
    int gap_ok = 1;
    for (int i = 0; i < e->path_len; ++i) gap_ok &= gaps[e->path[i][0] * RD + e->path[i][1]] != 1;
    uint8_t onpath[RD][RD];
    memset(onpath, 0, sizeof(onpath));
    for (int i = 0; i < e->path_len; ++i) onpath[e->path[i][0]][e->path[i][1]] = 1;
    /* per region: colors over every symbol (_collect_region_symbols), squares, stars */
    static int32_t rcol[RD * RD][9];
    static uint8_t has_star[RD * RD], sq_bad[RD * RD];
    for (int r = 0; r < R.nreg; ++r) memset(rcol[r], 0, sizeof(rcol[r]));
    int dot_ok = 1, sq_ok = 1, star_ok = 1, tri_ok = 1, poly_layer = -1;
    for (int l = 0; l < NL; ++l) {
        const int kind = rp->layer_kind[L0 + l];
        const uint8_t *pl = rp->layers + (size_t)(L0 + l) * RD * RD;
        if (kind == L_POLY) poly_layer = L0 + l;
        for (int x = 0; x < H; ++x)
            for (int y = 0; y < W; ++y) {
                if (pl[x * RD + y] != 1) continue;
                if (kind == L_DOT && !onpath[x][y]) dot_ok = 0;   /* all_dots_collected 519-531 */
                const int rid = R.map[x][y];
                if (rid < 0) continue;
                const int c = col[x * RD + y];
                if (c) rcol[rid][c < 9 ? c : 0]++;
            }
    }
    /* square_color_separation 533-551 and star_pairing_exact 553-619 */
    for (int r = 0; r < R.nreg; ++r) has_star[r] = 0, sq_bad[r] = 0;
    for (int l = 0; l < NL; ++l) {
        const int kind = rp->layer_kind[L0 + l];
        if (kind != L_SQUARE && kind != L_STAR) continue;
        const uint8_t *pl = rp->layers + (size_t)(L0 + l) * RD * RD;
        for (int r = 0; r < R.nreg; ++r) {
            int colors = 0, nstar[9] = {0};
            int any = 0;
            for (int x = 1; x < H; x += 2)
                for (int y = 1; y < W; y += 2) {
                    if (R.map[x][y] != r || pl[x * RD + y] != 1) continue;
                    any = 1;
                    const int c = col[x * RD + y];
                    if (kind == L_SQUARE) {
                        if (c) colors |= 1 << c;
                    } else if (c == 0) {
                        star_ok = 0;
                    } else {
                        nstar[c < 9 ? c : 0]++;
                    }
                }
            if (!any) continue;
            if (kind == L_SQUARE) {
                if (__builtin_popcount(colors) > 1) sq_ok = 0;
            } else {
                for (int c = 1; c < 9; ++c)
                    if (nstar[c] && rcol[r][c] != 2) star_ok = 0;
            }
        }
    }
    /* triangles_edge_count 622-646 (interior cells, positive counts) */
    for (int l = 0; l < NL; ++l) {
        if (rp->layer_kind[L0 + l] != L_TRIANGLE) continue;
        const uint8_t *pl = rp->layers + (size_t)(L0 + l) * RD * RD;
        for (int x = 1; x < H - 1; ++x)
            for (int y = 1; y < W - 1; ++y) {
                if (pl[x * RD + y] != 1 || add[x * RD + y] <= 0) continue;
                const int t = onpath[x + 1][y] + onpath[x - 1][y] + onpath[x][y - 1] + onpath[x][y + 1];
                if (t != add[x * RD + y]) tri_ok = 0;
            }
    }
    /* poly_ylop_area 648-709: instances = additional_info values naming a polyshape */
    int poly_ok = 1;
    static piece_t polys[RD * RD][64], ylops[RD * RD][64];
    static int np[RD * RD], nyl[RD * RD];
    for (int r = 0; r < R.nreg; ++r) np[r] = nyl[r] = 0;
    int ninst = 0;
    const int S0 = rp->shape_first[q], NS = rp->shape_count[q];
    for (int x = 0; x < H; ++x)
        for (int y = 0; y < W; ++y) {
            const int64_t v = add[x * RD + y];
            if (v == 0) continue;
            int s = -1;
            for (int k = 0; k < NS; ++k)
                if (rp->shape_name[S0 + k] == v) { s = S0 + k; break; }
            if (s < 0) continue;
            if (poly_layer < 0) return -1;   /* self.obs_array['poly'] KeyError (734) */
            ++ninst;
            const int rid = R.map[x][y];
            if (rid < 0) continue;
            piece_t pc = {rp->shape_ncell[s], rp->shape_off + (size_t)s * RMAXSHAPE * 2, v};
            if (rp->layers[(size_t)poly_layer * RD * RD + x * RD + y] == 1) {
                if (np[rid] < 64) polys[rid][np[rid]++] = pc;
            } else {
                if (nyl[rid] < 64) ylops[rid][nyl[rid]++] = pc;
            }
        }
    if (ninst)
        for (int r = 0; r < R.nreg; ++r) {
            if (!np[r] && !nyl[r]) continue;
            int pa = 0, ya = 0;
            for (int i = 0; i < np[r]; ++i) pa += polys[r][i].n;
            for (int i = 0; i < nyl[r]; ++i) ya += ylops[r][i].n;
            const int ok = R.area[r] == pa - ya && polyfit_exact(&R, r, polys[r], np[r], ylops[r], nyl[r]);
            poly_ok &= ok;
        }
    int bits = reached | (!crossing) << 1 | gap_ok << 2 | dot_ok << 3 | sq_ok << 4 | star_ok << 5 |
               tri_ok << 6 | poly_ok << 7;
    if ((bits & 0xFF) == 0xFF) bits |= 1 << 8;
    return bits;
}

/* The c3r CPU baseline: oracle_step + the audit `audits` times per env-step (the reference's
 * step() runs _validate_rules at 1227 and again in _get_info 1011), next-step autoreset onto the
 * next puzzle (the reset step: _load_puzzle 182 and _get_info 1011), counter-hash random actions;
 * one env.  Returns the env-steps run in `steps`; *bits_xor folds every audit's bits (so the work
 * cannot be dropped). */
int64_t oracle_rules_rollout(const oracle_pool *pool, const oracle_rules_pool *rp, oracle_env *e, int64_t steps,
                             uint64_t seed, int traceback, int max_steps, int audits, int32_t *bits_xor) {
    int32_t acc = 0;
    int pending = 0;
    for (int64_t t = 0; t < steps; ++t) {
        if (pending) {
            oracle_reset(pool, e, (e->pid + 1) % pool->n_puzzles);
            pending = 0;
        } else {
            int8_t code;
            uint8_t fl;
            oracle_step(pool, e, (int)oracle_rand_action(seed, 0, (uint64_t)t), traceback, max_steps, &code, &fl);
            pending = (fl & 3) != 0;
        }
        for (int a = 0; a < audits; ++a) acc ^= oracle_rules_bits(rp, e->pid, e) + a;
    }
    *bits_xor = acc;
    return steps;
}
