/* sparc_oracle.c — CPU restatement of the SPaRC-Gym step path.  TEST INFRASTRUCTURE ONLY
 * (see sparc_oracle.h).  Every function cites the reference lines it restates:
 * /root/reference/SPaRC_Gym/SPaRC_Gym.py.  Pinned by tests/golden/*.json.gz.
 */
#include "sparc_oracle.h"
#include <string.h>

/* _action_to_direction, SPaRC_Gym.py:212-217: right, up, left, down on [x, y] */
static const int DX[4] = {1, 0, -1, 0};
static const int DY[4] = {0, -1, 0, 1};

int oracle_env_size(void) { return (int)sizeof(oracle_env); }

static inline const int32_t *dims_of(const oracle_pool *p, int pid) { return p->dims + 6 * pid; }
static inline int gap_at(const oracle_pool *p, int pid, int x, int y) {
    return p->gaps[(size_t)pid * ORACLE_MAXDIM * ORACLE_MAXDIM + x * ORACLE_MAXDIM + y] != 0;
}
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* _load_puzzle state init, SPaRC_Gym.py:166-187 (fresh planes: first-load semantics) */
int oracle_reset(const oracle_pool *pool, oracle_env *e, int pid) {
    if (pid < 0 || pid >= pool->n_puzzles) return -1;
    const int32_t *d = dims_of(pool, pid);
    memset(e, 0, sizeof(*e));
    e->pid = pid;
    e->x = d[2];
    e->y = d[3];
    e->path_len = 1;
    e->path[0][0] = d[2];
    e->path[0][1] = d[3];
    e->visited[d[2]][d[3]] = 1;   /* 185 */
    return 0;
}

/* _get_legal_actions, SPaRC_Gym.py:1024-1051, restated literally including np.clip (1037) */
int oracle_legal(const oracle_pool *pool, const oracle_env *e, int traceback) {
    const int32_t *d = dims_of(pool, e->pid);
    int X = d[0], Y = d[1], mask = 0;
    for (int a = 0; a < 4; ++a) {
        int nx = e->x + DX[a], ny = e->y + DY[a];
        int cx = clampi(nx, 0, X - 1), cy = clampi(ny, 0, Y - 1);
        if (gap_at(pool, e->pid, cx, cy)) continue;                        /* 1039 */
        if (e->visited[cx][cy] == 1) {                                       /* 1040 */
            if (traceback && e->path_len >= 2) {                             /* 1041-1042 */
                int lx = e->path[e->path_len - 2][0], ly = e->path[e->path_len - 2][1];
                if (lx == cx && ly == cy && nx == cx && ny == cy) mask |= 1 << a;  /* 1044-1046 */
            }
        } else if (nx == cx && ny == cy) {                                   /* 1048 */
            mask |= 1 << a;
        }
    }
    return mask;
}

/* np.array_equal(self.path, solution) (1206) and _is_on_solution_path (1244-1265) */
static int path_equals(const oracle_pool *p, const oracle_env *e, int s) {
    if (e->path_len != p->sol_len[s]) return 0;
    const int32_t *q = p->pts + 2 * (size_t)p->sol_off[s];
    for (int i = 0; i < e->path_len; ++i)
        if (e->path[i][0] != q[2 * i] || e->path[i][1] != q[2 * i + 1]) return 0;
    return 1;
}
static int path_is_prefix(const oracle_pool *p, const oracle_env *e, int s) {
    if (e->path_len > p->sol_len[s]) return 0;                               /* 1257 */
    const int32_t *q = p->pts + 2 * (size_t)p->sol_off[s];
    for (int i = 0; i < e->path_len; ++i)                                    /* 1261-1263 */
        if (e->path[i][0] != q[2 * i] || e->path[i][1] != q[2 * i + 1]) return 0;
    return 1;
}

/* step(), SPaRC_Gym.py:1111-1238 minus the info-only rule audit / render */
int oracle_step(const oracle_pool *pool, oracle_env *e, int action, int traceback, int max_steps,
                int8_t *code, uint8_t *flags) {
    const int32_t *d = dims_of(pool, e->pid);
    int ox = e->x, oy = e->y;                                                /* 1131 */
    if (e->step < 0x7fffffff) e->step += 1;                                  /* 1132 */
    int normal = 0;                                                          /* 1133 (x100) */
    int truncated = e->step >= max_steps;                                    /* 1134 */
    int legal = oracle_legal(pool, e, traceback);
    if (action >= 0 && action < 4 && ((legal >> action) & 1)) {              /* 1137 */
        int nx = e->x + DX[action], ny = e->y + DY[action];                  /* 1138-1139 */
        if (e->visited[nx][ny] == 1) {                                       /* 1141 */
            if (traceback) {
                int lx = e->path[e->path_len - 2][0], ly = e->path[e->path_len - 2][1];
                if (lx == nx && ly == ny) {                                  /* 1143-1166 */
                    e->visited[e->x][e->y] = 0;
                    e->x = nx; e->y = ny;
                    e->visited[nx][ny] = 1;
                    e->path_len -= 1;
                }
            }
        } else {                                                             /* 1167-1188 */
            e->x = nx; e->y = ny;
            e->visited[nx][ny] = 1;
            if (e->path_len < ORACLE_MAXPATH) {
                e->path[e->path_len][0] = nx;
                e->path[e->path_len][1] = ny;
                e->path_len += 1;
            }
        }
    }
    int terminated = (e->x == d[4] && e->y == d[5]);                         /* 1192 */
    int legal_after = oracle_legal(pool, e, traceback);
    if (legal_after == 0) truncated = 1;                                     /* 1195-1196 */
    if (terminated) truncated = 0;                                           /* 1198-1199 */
    int nsol = pool->sol_count[e->pid], s0 = pool->sol_first[e->pid];
    if (terminated || truncated) {                                           /* 1204-1213 */
        for (int i = 0; i < nsol; ++i) {
            if (path_equals(pool, e, s0 + i)) { e->outcome = 1; normal = 100; break; }
        }
        if (e->outcome != 1) { e->outcome = -1; normal = -100; }
    } else {                                                                 /* 1214-1223 */
        e->outcome = 0;
        if (!(ox == e->x && oy == e->y)) {
            for (int i = 0; i < nsol; ++i) {
                if (path_is_prefix(pool, e, s0 + i)) { normal = 1; break; }
                normal = -1;
            }
        }
    }
    *code = (int8_t)normal;
    *flags = (uint8_t)(terminated | (truncated << 1) | (legal_after << 2));
    return 0;
}

/* counter-based random action; must equal sparc_rand_action() in include/sparc_gym_amd.h */
uint32_t oracle_rand_action(uint64_t seed, uint64_t env, uint64_t t) {
    uint64_t z = seed + env * 0x9E3779B97F4A7C15ull + t * 0xD1B54A32D192ED03ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 62);
}

int oracle_rollout(const oracle_pool *pool, int n, oracle_env *envs, int T, const uint8_t *actions,
                   uint64_t seed, uint64_t env_offset, uint64_t t0, int traceback, int max_steps,
                   int autoreset, int8_t *rew, uint8_t *flags, int32_t *stats) {
    return oracle_rollout_obs(pool, n, envs, T, actions, seed, env_offset, t0, traceback, max_steps, autoreset,
                              rew, flags, stats, NULL, NULL, 0, 0);
}

/* obs['base']['visited'] / ['agent_location'] of env e as int32 planes [xd][yd] (_get_obs,
 * SPaRC_Gym.py:956-979; zero outside the puzzle's lattice) */
static void write_planes(const oracle_env *e, int32_t *vis, int32_t *agent, int xd, int yd) {
    for (int x = 0; x < xd; ++x)
        for (int y = 0; y < yd; ++y) {
            int inb = x < ORACLE_MAXDIM && y < ORACLE_MAXDIM;
            if (vis) vis[x * yd + y] = inb ? e->visited[x][y] : 0;
            if (agent) agent[x * yd + y] = (x == e->x && y == e->y);
        }
}

int oracle_rollout_obs(const oracle_pool *pool, int n, oracle_env *envs, int T, const uint8_t *actions,
                       uint64_t seed, uint64_t env_offset, uint64_t t0, int traceback, int max_steps,
                       int autoreset, int8_t *rew, uint8_t *flags, int32_t *stats, int32_t *vis,
                       int32_t *agent, int xd, int yd) {
    const size_t plane = (size_t)xd * yd;
    for (int i = 0; i < n; ++i) {
        oracle_env *e = &envs[i];
        for (int t = 0; t < T; ++t) {
            int8_t c = 0;
            uint8_t f = 0;
            if (autoreset == 1 && e->pending) {
                /* gymnasium next-step autoreset: reset() picks the next puzzle (SPaRC_Gym.py:1087) */
                oracle_reset(pool, e, (e->pid + 1) % pool->n_puzzles);
                f = (uint8_t)((oracle_legal(pool, e, traceback) << 2) | 0x40);
                if (stats) stats[4 * i + 3] += 1;
            } else {
                int a = actions ? actions[(size_t)t * n + i]
                                : (int)oracle_rand_action(seed, env_offset + i, t0 + t);
                oracle_step(pool, e, a, traceback, max_steps, &c, &f);
                e->pending = (f & 3) != 0;
                if (stats) {
                    stats[4 * i + 0] += c;
                    if (f & 3) { stats[4 * i + 1] += 1; if (c == 100) stats[4 * i + 2] += 1; }
                }
            }
            if (rew) rew[(size_t)t * n + i] = c;
            if (flags) flags[(size_t)t * n + i] = f;
            if (vis || agent)
                write_planes(e, vis ? vis + ((size_t)t * n + i) * plane : NULL,
                             agent ? agent + ((size_t)t * n + i) * plane : NULL, xd, yd);
        }
    }
    return 0;
}
