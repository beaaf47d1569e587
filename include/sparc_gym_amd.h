/* sparc_gym_amd.h — C ABI of the MI355X-native batched SPaRC step path.
 *
 * The reference (tobiTKM/SPaRC-Gym) is pure Python: one `SPaRC_Gym(gym.Env)` object holds one
 * puzzle and `step(action)` runs on host numpy.  It has no FFI, so the entry points below are
 * the C ABI its step path would bind through ctypes; each one cites the reference code it
 * replaces (/root/reference/SPaRC_Gym/SPaRC_Gym.py).  The Python host layer in
 * sparc-gym_amd/sparc_gym_amd/ (SPaRC_Gym, SPaRCVecEnv) binds exactly these symbols.
 *
 * Conventions
 *  - Plain pointers and sizes; no torch / HIP types in the signatures (streams are void*).
 *  - Every call returns SPARC_OK (0) or a negative error code; the message is available from
 *    sparc_last_error(ctx) (or sparc_last_error(NULL) after a failed sparc_create).  No C++
 *    exception crosses the ABI.
 *  - `*_device` / rollout entry points take DEVICE pointers and are asynchronous on the
 *    context's stream.  `*_host` entry points take host pointers and return after the data are
 *    back on the host.
 *  - One context per GPU, not reentrant; all work is ordered on its stream.
 *
 * Lattice encoding: planes are indexed [x, y] with x_size = 2*width+1, y_size = 2*height+1
 * (SPaRC_Gym.py:243-248).  A point is bit b = x*pitch + y of a `words`-word bitboard.
 *  words == 1: padded layout, every puzzle has y_size < pitch <= 15 and
 *              (x_size + 1) * pitch <= 64 (7x7 / 5x5 pools; the kernels' fast path);
 *  words 2, 4: pitch >= every y_size and (x_size - 1) * pitch + y_size <= 64 * words.
 *
 * Per-step outputs
 *  reward code  int8  = normal_reward * 100: {-100, -1, 0, +1, +100}  (SPaRC_Gym.py:1201-1223);
 *                       the host maps it back to the reference's Python values
 *                       {-1 (int), -0.01, 0 (int), 0.01, 1 (int)}.
 *  flags        uint8 bit0 terminated, bit1 truncated (SPaRC_Gym.py:1192-1199),
 *                     bits2-5 legal actions after the step (info['legal_actions'], 1016),
 *                     bit6 this step was an autoreset (gymnasium next-step mode).
 *  outcome_reward (info['Rewards'], 1020) = done ? (code==-100 ? -1 : 1) : 0.
 */
#ifndef SPARC_GYM_AMD_H
#define SPARC_GYM_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPARC_ABI_VERSION 2

enum {
    SPARC_OK = 0,
    SPARC_E_INVALID = -1,   /* bad argument / shape / puzzle index              */
    SPARC_E_HIP = -2,       /* HIP runtime error                                  */
    SPARC_E_STATE = -3,     /* call order (e.g. step before load_puzzles/reset)   */
    SPARC_E_NOMEM = -4,
    SPARC_E_COMM = -5       /* RCCL unavailable or a collective failed            */
};

enum { SPARC_AUTORESET_NONE = 0, SPARC_AUTORESET_NEXT_STEP = 1 };

enum {
    SPARC_FLAG_TERMINATED = 1,
    SPARC_FLAG_TRUNCATED = 2,
    SPARC_FLAG_LEGAL_SHIFT = 2,
    SPARC_FLAG_RESET = 64
};

/* Constructor kwargs of SPaRC_Gym.__init__ (SPaRC_Gym.py:46) that reach the step path, plus
 * the batch shape.  The dataset kwargs (df_name/df_split/df_set) stay in the host layer. */
typedef struct {
    int32_t num_envs;
    int32_t traceback;      /* SPaRC_Gym.py:65, 1041-1046, 1142-1166                      */
    int32_t max_steps;      /* SPaRC_Gym.py:66, 1134                                      */
    int32_t autoreset;      /* SPARC_AUTORESET_*; NONE reproduces the reference exactly   */
    int32_t pitch;          /* bitboard row pitch (>= max y_size)                         */
    int32_t words;          /* bitboard words: 1, 2 or 4                                  */
    int64_t env_offset;     /* global id of env 0 (multi-GPU shards; random actions)      */
} sparc_config;

/* Static puzzle table, packed by the host loader (sparc_gym_amd/puzzles.py) from the
 * processed puzzles of _process_puzzles (SPaRC_Gym.py:219-368).
 *  open  [P][words]  bit set = lattice point inside the puzzle and gaps[x][y] == 0
 *  info  [P][4]      w0 = x_size | y_size<<8 | start_x<<16 | start_y<<24
 *                    w1 = target_x | target_y<<8 | flags<<16
 *                         (flags bit0: solution_count > 0, bit1: some solution starts at start,
 *                          bit2: the start point is a gap)
 *                    w2 = global index of the puzzle's trie root, w3 = its trie node count
 *  trie  [nodes][4]  solution-prefix trie, local (per puzzle) u16 indices, 0xFFFF = none:
 *                    w0 = child[right] | child[up]<<16, w1 = child[left] | child[down]<<16,
 *                    w2 = parent | terminal<<16 | child_terminal[4]<<17 | parent_terminal<<21,
 *                    w3 = depth.  Node 0 of each puzzle is the one-point path [start].      */
typedef struct {
    int32_t num_puzzles;
    int32_t num_nodes;
    const uint64_t *open;
    const uint32_t *info;
    const uint32_t *trie;
} sparc_puzzle_table;

/* Host snapshot of the per-env state (any pointer may be NULL to skip that field). */
typedef struct {
    uint8_t *x, *y;         /* _agent_location              [N] */
    uint16_t *path_len;     /* len(self.path)               [N] */
    uint32_t *step;         /* current_step                 [N] */
    uint32_t *puzzle;       /* current_puzzle_index         [N] */
    int8_t *outcome;        /* outcome_reward               [N] */
    uint8_t *pending;       /* done on the last step        [N] */
    uint64_t *visited;      /* obs['base']['visited'] bits  [words][N] */
} sparc_state_host;

/* counter-based random action in {0,1,2,3} (splitmix64 finaliser of seed, env, t); stands in
 * for env.action_space.sample() (Final_Product.py:29) in device rollouts. */
static inline uint32_t sparc_rand_action(uint64_t seed, uint64_t env, uint64_t t) {
    uint64_t z = seed + env * 0x9E3779B97F4A7C15ull + t * 0xD1B54A32D192ED03ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 62);
}

int sparc_abi_version(void);
const char *sparc_last_error(const void *ctx);

/* SPaRC_Gym.__init__ (SPaRC_Gym.py:46-90): allocate the SoA state for num_envs on `device`. */
int sparc_create(int device, const sparc_config *cfg, void **ctx_out);
int sparc_destroy(void *ctx);
/* run on this HIP stream (hipStream_t as void*; NULL = the HIP null stream).  A new context
 * runs on its own non-blocking stream; sparc_use_own_stream() returns to it. */
int sparc_set_stream(void *ctx, void *stream);
int sparc_use_own_stream(void *ctx);
int sparc_sync(void *ctx);

/* _process_puzzles output -> device (SPaRC_Gym.py:88, 219-368); host arrays, copied. */
int sparc_load_puzzles(void *ctx, const sparc_puzzle_table *table);

/* reset / _load_puzzle (SPaRC_Gym.py:1057-1108, 141-187) for every env with mask[i] != 0
 * (mask NULL = all) onto puzzle puzzle_index[i].  Arrays of length num_envs.  flags (may be
 * NULL) receives, for the reset envs, the legal actions of the fresh state in bits 2-5 —
 * info['legal_actions'] of reset()'s _get_info (SPaRC_Gym.py:1016, 1108). */
int sparc_reset_host(void *ctx, const uint32_t *puzzle_index, const uint8_t *mask, uint8_t *flags);
int sparc_reset_device(void *ctx, const uint32_t *d_puzzle_index, const uint8_t *d_mask, uint8_t *d_flags);

/* step (SPaRC_Gym.py:1111-1238) for all envs: one action per env (values >= 4 are illegal
 * and leave the agent in place, as `action in legal` fails at 1137). */
int sparc_step_device(void *ctx, const uint8_t *d_actions, int8_t *d_reward, uint8_t *d_flags);
int sparc_step_host(void *ctx, const uint8_t *actions, int8_t *reward, uint8_t *flags);

/* T consecutive steps in ONE launch (state stays in registers): actions [T][N] device
 * (or NULL: sparc_rand_action(seed, env_offset+i, t0+t)); reward/flags [T][N] device (may be
 * NULL); stats [N][4] int32 device, accumulated: {sum of reward codes, done steps,
 * solved (+1) steps, autoresets} (may be NULL).  Bit-identical to T sparc_step_device calls. */
int sparc_rollout_device(void *ctx, int32_t T, const uint8_t *d_actions, uint64_t seed, uint64_t t0,
                         int8_t *d_reward, uint8_t *d_flags, int32_t *d_stats);

/* env.action_space.sample() (Final_Product.py:29) for every env and T steps, into HBM:
 * d_actions [T][N] uint8, entry (t, i) = sparc_rand_action(seed, env_offset+i, t0+t) — the
 * actions a NULL-action rollout draws, seeded by the GLOBAL env id so that the shards of a
 * multi-GPU job hold exactly the actions of one process over all envs.  Asynchronous. */
int sparc_random_actions_device(void *ctx, int32_t T, uint64_t seed, uint64_t t0, uint8_t *d_actions);

/* obs['base']['visited'] / obs['base']['agent_location'] as dense int32 planes
 * [N][x_dim][y_dim] (x_dim >= max x_size, y_dim >= max y_size; device pointers, either may be
 * NULL).  The reference returns these planes by reference every step (SPaRC_Gym.py:979). */
int sparc_obs_pack_device(void *ctx, int32_t *d_visited, int32_t *d_agent, int32_t x_dim, int32_t y_dim);

/* step (SPaRC_Gym.py:1111-1238) and the 'new' observation it returns (_get_obs 956-979) in ONE
 * launch: reward/flags as sparc_step_device, then the post-step visited / agent_location
 * planes [N][x_dim][y_dim] int32 (either may be NULL), the current puzzle index [N] (after any
 * autoreset; may be NULL) and the agent location [N] = x | y << 8 (may be NULL).
 * x_dim * y_dim <= 256.  Device pointers, asynchronous. */
int sparc_step_obs_device(void *ctx, const uint8_t *d_actions, int8_t *d_reward, uint8_t *d_flags,
                          int32_t *d_visited, int32_t *d_agent, int32_t x_dim, int32_t y_dim,
                          uint32_t *d_puzzle, uint32_t *d_xy);

/* One gymnasium vector step in ONE launch (SPaRCVecEnv.step; SPaRC_Gym.step 1111-1238 for every
 * env): the step and its 'new' planes as sparc_step_obs_device, plus the gym outputs the host
 * would otherwise derive with separate launches:
 *   d_actions: [N] elements of action_bytes = 1 (uint8; >= 4 is illegal = no move), 4 (int32)
 *              or 8 (int64; < 0 or >= 4 is illegal), so a caller's int64 actions need no cast;
 *   d_reward [N] double = reward code / 100 (the reference's exact float64 values -1, -0.01,
 *   0, 0.01, 1); d_terminated / d_truncated / d_autoreset [N] 0/1 bytes (bool tensors);
 *   d_legal [N] = the legal-action mask of the new state (bit a = action a, 1024-1051);
 *   d_loc [N][2] int32 = the agent's (x, y).
 * Every output pointer may be NULL (not written).  x_dim * y_dim <= 256 when planes are given.
 * Device pointers, asynchronous. */
int sparc_step_gym_device(void *ctx, const void *d_actions, int32_t action_bytes, double *d_reward,
                          uint8_t *d_terminated, uint8_t *d_truncated, uint8_t *d_legal, uint8_t *d_autoreset,
                          int8_t *d_reward_code, uint8_t *d_flags, int32_t *d_visited, int32_t *d_agent,
                          int32_t x_dim, int32_t y_dim, uint32_t *d_puzzle, int32_t *d_loc);

/* sparc_rollout_device that also records the 'new' observation after every step: planes
 * [T][N][x_dim][y_dim] int32 (visited / agent_location; either may be NULL), so step t's
 * entries equal sparc_step_obs_device's after the t-th of T single steps.  Every store is a
 * whole 16-B piece of a contiguous per-wave run when N * x_dim * y_dim % 4 == 0 and the
 * pointers are 16-B aligned.  x_dim * y_dim <= 256.  This mode is HBM-write-bound
 * (8 * x_dim * y_dim bytes per env-step). */
int sparc_rollout_obs_device(void *ctx, int32_t T, const uint8_t *d_actions, uint64_t seed, uint64_t t0,
                             int8_t *d_reward, uint8_t *d_flags, int32_t *d_stats, int32_t *d_visited,
                             int32_t *d_agent, int32_t x_dim, int32_t y_dim);

/* sparc_rollout_device that also runs the rule audit after every step, as the reference's
 * step() does (_validate_rules at SPaRC_Gym.py:1227 and again in _get_info 1011, filling
 * info['rule_status'], 941-950): d_rule_bits [T][N] uint16, step t's entry equal to
 * sparc_rules_device's bits after the t-th of T single steps.  Needs sparc_load_rules.  The
 * audit (flood fills, exact-fit searches) costs far more than the step.  On one-word (5x5 /
 * 7x7) pools whose every puzzle has a region-code table this runs k_rollout1r (per 64 envs a
 * step wave and five audit waves); otherwise the generic per-wave rule kernel.  The bits are
 * identical. */
int sparc_rollout_rules_device(void *ctx, int32_t T, const uint8_t *d_actions, uint64_t seed, uint64_t t0,
                               int8_t *d_reward, uint8_t *d_flags, int32_t *d_stats, uint16_t *d_rule_bits);

int sparc_read_state(void *ctx, const sparc_state_host *out);

/* ---- one env in one round trip: the drop-in SPaRC_Gym (a context of one env) -----------------
 * Everything SPaRC_Gym.step() / reset() returns for env `env` of the context, written by the
 * kernels straight into a pinned record and read back with ONE stream synchronisation: the step's
 * reward code and flags, the new state, and (audit != 0, after sparc_load_rules) the rule audit of
 * the new state with its region ids and fit mask (info['rule_status'], _validate_rules 941-950).
 * An exact fit past the GPU's node cap (rare) is finished on the host before the call returns, so
 * rule_bits never holds SPARC_RULE_SEARCH_EXHAUSTED (one more synchronisation, that call only).
 * The audit covers every env of the context (k_rules): meant for contexts of one env. */
typedef struct {
    int8_t reward_code;     /* the step's reward * 100 (0 after reset / read), SPaRC_Gym.py:1201-1223 */
    uint8_t flags;          /* bit0 terminated, bit1 truncated, bits2-5 legal actions of the new state */
    uint8_t x, y;           /* _agent_location                                                       */
    uint8_t path_len;       /* len(self.path)                                                        */
    int8_t outcome;         /* outcome_reward (info['Rewards'], 1020)                                */
    uint8_t pending;        /* the last step was done (next-step autoreset pending)                 */
    uint8_t audited;        /* 1: rule_bits / fit / region below are the new state's audit         */
    uint32_t step;          /* current_step                                                          */
    uint32_t puzzle;        /* current_puzzle_index                                                  */
    uint16_t rule_bits;     /* SPARC_RULE_*                                                          */
    uint16_t reserved;
    uint32_t host_fits;     /* exact fits of this audit the host finished (0 on nearly every call)  */
    uint64_t fit;           /* bit r: region r passed the poly/ylop area check and exact fit        */
    uint64_t visited[4];    /* obs['base']['visited'] bits x*pitch + y (the first `words` words)    */
    uint8_t region[256];    /* region id per cell bit (64 * words entries), 0xFF elsewhere          */
} sparc_env_record;
/* step (SPaRC_Gym.py:1111-1238) of env `env` with `action` (outside 0..3: illegal, no move) */
int sparc_env_step(void *ctx, int32_t env, int32_t action, int32_t audit, sparc_env_record *out);
/* reset / _load_puzzle (1057-1108, 95-217) of env `env` onto puzzle `puzzle_index` */
int sparc_env_reset(void *ctx, int32_t env, uint32_t puzzle_index, int32_t audit, sparc_env_record *out);
/* the current state (and audit) of env `env`, no transition */
int sparc_env_read(void *ctx, int32_t env, int32_t audit, sparc_env_record *out);
/* device-to-device copy of one SoA state array (`which` as in sparc_state_ptr) into d_out,
 * ordered on the context's stream (e.g. the per-env puzzle index after autoresets). */
int sparc_copy_state_device(void *ctx, int32_t which, void *d_out);

/* Overwrite the visited boards [words][N] (host, bit x*pitch+y) of the current state, e.g. with
 * the planes an aliasing reference env keeps across re-loads of a puzzle (SPaRC_Gym.py:149-151:
 * _load_puzzle binds the puzzle's planes, so a re-loaded puzzle starts with the previous
 * episode's visited bits, which _get_legal_actions (1040) and step (1141) then read).  Every
 * env's board must hold its start point (visited[start] = 1, SPaRC_Gym.py:185) and no bit
 * outside its puzzle's lattice, else SPARC_E_INVALID and the state is unchanged.  Synchronous. */
int sparc_set_visited_host(void *ctx, const uint64_t *visited);

/* device pointers of the context's SoA state (zero-copy views for the host layer):
 * which: 0 visited [words][N] u64, 1 pos [N] u32 = x | y<<8 | len<<16 | off<<24,
 *        2 aux [N] u32 = trie node | outcome<<16 (1: +1, 2: -1) | pending<<18,
 *        3 step [N] u32, 4 puzzle [N] u32, 5 direction stack [2*words][N] u64 (traceback) */
int sparc_state_ptr(void *ctx, int32_t which, void **d_ptr);

/* ---- rule audit: info['rule_status'] (_validate_rules, SPaRC_Gym.py:941-950) ----------------
 * Rule table, packed by sparc_gym_amd/puzzles.py:pack_rules from the processed puzzles, on the
 * step table's geometry (bit x*pitch + y, `words` u64 per board).
 *  planes      [P][SPARC_RULE_PLANES][words]: cells (odd, odd), lattice, gaps, dots, triangle
 *              cells with count > 0 (x in 1..x_size-2, y in 1..y_size-2) and their count bits
 *              0-2 (count clamped to 7), star, square, coloured, colour 1..8, per-cell symbol
 *              multiplicity bits 0-2 (layers other than visited/gaps/agent/target set at a
 *              cell), y != 0, y != y_size-1, cells holding a poly/ylop instance
 *  inst_first  [P + 1] offsets into inst: puzzle q's poly/ylop instances (at cell centres,
 *              _extract_poly_instances 714-734) are inst[inst_first[q] .. inst_first[q + 1])
 *  inst        bit | ylop << 10 | shape << 11 (shape < 2^21)
 *  shape_first [S + 1] offsets into shape_off: shape s's cells are shape_off[shape_first[s] ..
 *              shape_first[s + 1]), (dx, dy) in cell units relative to the shape's anchor
 *              (_get_offsets 840-855); shape_area [S] = sum of the shape array (722)
 * No pool-wide limit.  Lattices up to 15 x 15.  The exact-fit searches of a puzzle with more
 * than 16 ylops or 16 distinct poly shapes (its instances' lists outgrow the GPU search's) run
 * on the host (sparc_rules_finish), with the same search code; every answer is the same.      */
#define SPARC_RULE_PLANES 25
typedef struct {
    int32_t num_puzzles;    /* must equal the loaded step table's */
    int32_t num_inst;
    int32_t num_shapes;
    int32_t num_offsets;
    const uint64_t *planes;
    const uint32_t *inst_first;
    const uint32_t *inst;
    const uint32_t *shape_first;
    const int32_t *shape_area;
    const int8_t *shape_off;
} sparc_rules_table;

enum {
    SPARC_RULE_REACHED_TARGET = 1 << 0,       /* _rule_reached_target 487-495        */
    SPARC_RULE_PATH_NOT_CROSSING = 1 << 1,    /* 497-505                             */
    SPARC_RULE_NO_GAP_VIOLATIONS = 1 << 2,    /* 507-517                             */
    SPARC_RULE_ALL_DOTS_COLLECTED = 1 << 3,   /* 519-531                             */
    SPARC_RULE_SQUARE_SEPARATION = 1 << 4,    /* 533-551                             */
    SPARC_RULE_STAR_PAIRING = 1 << 5,         /* 553-619                             */
    SPARC_RULE_TRIANGLES = 1 << 6,            /* 622-646                             */
    SPARC_RULE_POLY_YLOP = 1 << 7,            /* 648-838                             */
    SPARC_RULE_ALL = 1 << 8,                  /* all_rules_satisfied 931-936         */
    /* not a rule: an exact-fit search of this audit (_polyfit_region_exact, 738-853) passed the
     * GPU's node cap (sparc_set_rule_limits; 2^26 by default) and is PENDING: its region counts
     * as passing until sparc_rules_finish has run the search to its end on the host (the
     * reference's search is unbounded) and patched POLY_YLOP / ALL.  Never set after
     * sparc_rules_finish (sparc_rules_host calls it itself). */
    SPARC_RULE_SEARCH_EXHAUSTED = 1 << 9
};

/* Load the rule table (host arrays, copied).  Call after sparc_load_puzzles, which drops it. */
int sparc_load_rules(void *ctx, const sparc_rules_table *table);
/* Audit the current state of every env: bits [N] (SPARC_RULE_*), and optionally
 * region [N][64*words] (region id of each cell bit in the reference's numbering, 0xFF
 * elsewhere) and fit [N] (bit r: region r holds poly/ylop instances and passes both the area
 * check and the exact fit).  Device pointers; any output may be NULL. */
int sparc_rules_device(void *ctx, uint16_t *d_bits, uint8_t *d_region, uint64_t *d_fit);
int sparc_rules_host(void *ctx, uint16_t *bits, uint8_t *region, uint64_t *fit);

/* Finish the exact-fit searches that passed the GPU's node cap (or belong to a puzzle whose
 * searches run on the host) in the LAST audit call (sparc_rules_device, or
 * sparc_rollout_rules_device: its d_rule_bits) on the host, without a cap, and patch that call's
 * outputs on the device: SPARC_RULE_SEARCH_EXHAUSTED cleared, POLY_YLOP and ALL cleared when a
 * region does not fit, and (d_fit, may be NULL) the fit bits of the regions that do.  Call it
 * after each such call, before reading its bits, with that call's output pointers, and before its
 * inputs change (a call that queued more searches than the queue holds is run again on a larger
 * queue, from the state, stats and memo it started from).  Synchronous (a 4-byte read when
 * nothing was queued).  SPARC_E_STATE: no audit call to finish, or bits of another call. */
int sparc_rules_finish(void *ctx, uint16_t *d_bits, uint64_t *d_fit);

/* out[3]: the exact-fit queue's capacity (65,536 entries at first, grown on overflow), the
 * searches the last sparc_rules_finish ran on the host, and the audit calls run again so far
 * because their searches overflowed the queue (diagnostics: how much of the audit went to the
 * host). */
int sparc_rules_queue_stats(void *ctx, uint64_t *out);

/* Limits of the rule audit: fit_cap_nodes = search nodes one exact fit runs on the GPU before the
 * host finishes it (0: 2^26); table_entries = the region-code table budget in 4-bit entries
 * (0: 2^28 = 128 MB; puzzles past it are audited by the memoised search instead).  The cap applies
 * to the following audits and the next sparc_load_rules, the budget to the next sparc_load_rules. */
int sparc_set_rule_limits(void *ctx, uint32_t fit_cap_nodes, uint64_t table_entries);

/* ---- debug: kernel variants (A/B runs and tests) ----------------------------------------------
 * Selects, for this context, among kernel variants that compute identical results.  Callers never
 * need it, and nothing else (no environment variable) changes the kernel a context runs.
 *  SPARC_VARIANT_IO_CODES_OFF          1: under next-step autoreset the split rollouts keep the
 *                                      reward codes on the trie wave (k_rollout1s / k_rolloutWs
 *                                      without the I/O-wave codes); 0: default
 *  SPARC_VARIANT_RULE_ROLLOUT_GENERIC  1: rule rollouts on the generic per-wave rule kernel even
 *                                      where k_rollout1r applies; 0: default
 *  SPARC_VARIANT_R1R_SHAPE             k_rollout1r's <G, A, RT>: 0 <2, 5, 15> (default),
 *                                      1 <4, 3, 12>, 2 <2, 4, 12>, 5 <2, 5, 10>; incremental
 *                                      audits (each audit wave keeps its envs' regions from
 *                                      step to step): 3 <4, 1, 4>, 4 <2, 3, 15>
 *  SPARC_VARIANT_OBS_INLINE            1: sparc_rollout_obs_device on the per-wave kernel that
 *                                      writes its own planes; 0: default (writer waves)
 *  SPARC_VARIANT_MIXED_TRIE            W = 1 pools past the LDS row budget: the split kernel on
 *                                      the mixed trie tables (4-B records for tries of <= 127
 *                                      nodes) 0: when the 8-B records outgrow 4 MB (default),
 *                                      1: always, 2: never
 *  SPARC_VARIANT_HOST_FITS             1: the answers of exact fits finished on the host are not
 *                                      kept for later audits (every such search is queued again:
 *                                      tests of the queue path); 0: default
 * SPARC_E_INVALID for another `which` or value. */
enum { SPARC_VARIANT_IO_CODES_OFF = 1, SPARC_VARIANT_RULE_ROLLOUT_GENERIC = 2, SPARC_VARIANT_R1R_SHAPE = 3,
       SPARC_VARIANT_OBS_INLINE = 4, SPARC_VARIANT_MIXED_TRIE = 5, SPARC_VARIANT_HOST_FITS = 6 };
int sparc_set_variant(void *ctx, int32_t which, int32_t value);

/* ---- multi-GPU: the end-of-batch gather over RCCL (xGMI) -------------------------------------
 * The envs shard across GPUs as contiguous global id ranges (env_offset), one process and one
 * context per GPU, no data-path collective; after a rollout batch the per-env stats are gathered
 * with ONE ncclAllGather (SURVEY.md §8b/§8e "sparc_rccl_gather").  The reference has no
 * counterpart: it is one env per process (SPaRC_Gym.py:44; llm_host.py:257-264 runs independent
 * envs concurrently).  librccl is opened on first use (SPARC_E_COMM when absent).
 *  sparc_comm_unique_id  rank 0 creates the rendezvous id (ncclGetUniqueId) and hands the
 *                        SPARC_COMM_ID_BYTES bytes to every rank over any channel it has;
 *  sparc_comm_init       every rank joins (ncclCommInitRank on the context's GPU; blocks until
 *                        all nranks have joined);
 *  sparc_gather_stats    d_stats [N][4] int32 of this rank (sparc_rollout_device's) ->
 *                        d_out [nranks][N][4] on every rank, ordered by rank = by global env id;
 *                        asynchronous on the context's stream, N equal on every rank. */
#define SPARC_COMM_ID_BYTES 128
int sparc_comm_unique_id(uint8_t *id_out);
int sparc_comm_init(void *ctx, int32_t nranks, int32_t rank, const uint8_t *id, void **comm_out);
int sparc_comm_destroy(void *comm);
int sparc_gather_stats(void *ctx, void *comm, const int32_t *d_stats, int32_t *d_out);

#ifdef __cplusplus
}
#endif
#endif
