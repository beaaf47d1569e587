/* sparc_oracle.h — CPU restatement of the SPaRC-Gym step path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is the parity checker for the HIP kernels, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It restates the
 * reference algorithm literally (path as a list of points, O(S*L) solution compares, the
 * np.clip legality trick) so that it shares no data structure with the GPU path (which
 * uses bitboards, a 2-bit direction stack and a solution trie).
 *
 * Reference: /root/reference/SPaRC_Gym/SPaRC_Gym.py
 *   _get_legal_actions  1024-1051      step              1111-1238
 *   _is_on_solution_path 1244-1265     reset/_load_puzzle 1057-1108, 141-187
 * Pinned by tests/golden/*.json.gz (generated from the reference itself).
 */
#ifndef SPARC_ORACLE_H
#define SPARC_ORACLE_H
#include <stdint.h>

#define ORACLE_MAXDIM 16            /* lattice x_size, y_size <= 16 */
#define ORACLE_MAXPATH 257

typedef struct {
    int32_t n_puzzles;
    const int32_t *dims;       /* [P][6]: x_size, y_size, start_x, start_y, target_x, target_y */
    const uint8_t *gaps;       /* [P][16][16] gaps plane (nonzero = gap), [x][y]               */
    const int32_t *sol_count;  /* [P] solution_count as used by range() (SPaRC_Gym.py:1205)    */
    const int32_t *sol_first;  /* [P] first solution of puzzle p in sol_len / sol_off           */
    const int32_t *sol_len;    /* [S] number of points                                         */
    const int32_t *sol_off;    /* [S] offset (in points) into pts                              */
    const int32_t *pts;        /* [n_pts][2] (x, y)                                             */
} oracle_pool;

typedef struct {
    int32_t x, y;              /* _agent_location                    */
    int32_t step;              /* current_step                        */
    int32_t outcome;           /* outcome_reward in {-1, 0, 1}        */
    int32_t pid;               /* current_puzzle_index                */
    int32_t path_len;
    int32_t pending;           /* done on the previous step (autoreset NEXT_STEP) */
    int32_t pad;
    int32_t path[ORACLE_MAXPATH][2];
    uint8_t visited[ORACLE_MAXDIM][ORACLE_MAXDIM];
} oracle_env;

#ifdef __cplusplus
extern "C" {
#endif
int oracle_env_size(void);
int oracle_reset(const oracle_pool *pool, oracle_env *e, int pid);
int oracle_legal(const oracle_pool *pool, const oracle_env *e, int traceback);
/* one reference step(); reward code = normal_reward * 100 in {-100,-1,0,1,100};
 * flags: bit0 terminated, bit1 truncated, bits2-5 legal actions after the step, bit6 reset */
int oracle_step(const oracle_pool *pool, oracle_env *e, int action, int traceback, int max_steps,
                int8_t *code, uint8_t *flags);
/* T steps of n envs; actions [T][n] (NULL -> counter-hash random actions from seed);
 * autoreset 0 = none (reference), 1 = next-step; stats [n][4] accumulated (may be NULL) */
int oracle_rollout(const oracle_pool *pool, int n, oracle_env *envs, int T, const uint8_t *actions,
                   uint64_t seed, uint64_t env_offset, uint64_t t0, int traceback, int max_steps,
                   int autoreset, int8_t *rew, uint8_t *flags, int32_t *stats);
/* oracle_rollout that also records the post-step visited / agent_location planes of every
 * step: [T][n][xd][yd] int32 (either may be NULL) */
int oracle_rollout_obs(const oracle_pool *pool, int n, oracle_env *envs, int T, const uint8_t *actions,
                       uint64_t seed, uint64_t env_offset, uint64_t t0, int traceback, int max_steps,
                       int autoreset, int8_t *rew, uint8_t *flags, int32_t *stats, int32_t *vis,
                       int32_t *agent, int xd, int yd);
uint32_t oracle_rand_action(uint64_t seed, uint64_t env, uint64_t t);
#ifdef __cplusplus
}
#endif
#endif
