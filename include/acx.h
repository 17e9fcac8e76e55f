/*
 * acx.h -- C-ABI of libacx.so, the MI355X (gfx950) Andrews-Curtis environment kernels.
 *
 * Drop-in boundary for the hot path of Avi161/AC-Solver-Caltech (reference paths are
 * relative to the reference repository root):
 *
 *   acx_step        replaces ACEnv.step            ac_solver/envs/ac_env.py:91-111
 *                   (ACMove ac_solver/envs/ac_moves.py:159-231 -> concatenate_relators
 *                    :4-76 | conjugate :79-156 -> simplify_presentation
 *                    ac_solver/envs/utils.py:246-283), batched over B envs, plus the
 *                   same-step autoreset gymnasium's SyncVectorEnv applies around it
 *                   (ac_solver/agents/environment.py:96-101, training.py:238-240).
 *                   With reward/done/truncated/step_count all NULL it is a batched
 *                   ACMove.
 *   acx_rollout     T fused ACEnv.step calls (the PPO rollout collection loop,
 *                   ac_solver/agents/training.py:221-356), state kept on chip.
 *   acx_expand12    the 12-way neighbour expansion of greedy_search / bfs
 *                   (ac_solver/search/greedy.py:202-210, breadth_first.py:69-77).
 *   acx_canonicalize  simplify_presentation (utils.py:246-283) over a batch.
 *   acx_unpack_keys   packed child keys (acx_expand12) -> int32 presentations.
 *
 * Conventions
 *   - A presentation is 2L int32 letters: relator r0 in [0,L), r1 in [L,2L); letters
 *     +-1 (x), +-2 (y); 0 is right padding (utils.py:1-8).  Batches are row-major (B,2L).
 *   - All pointers are device pointers (hipMalloc / torch CUDA tensors), 16-byte aligned.
 *     Every call is asynchronous on `stream` (a hipStream_t; NULL = default stream) and
 *     never allocates or synchronises, so it can be captured into a hipGraph.
 *   - Return value: ACX_OK, or a negative ACX_E_* status for bad arguments / a failed
 *     launch.  Per-env failures are reported in the optional `err` byte array with the
 *     ACX_ERR_* codes below; an env with err != 0 keeps its input state (the reference
 *     raises instead).  `err_count` (nullable, one int32) is atomically incremented once
 *     per env with err != 0, so the host can check one word instead of B bytes.
 *   - L (max_relator_length) must be in [1, ACX_MAX_L].
 */
#ifndef ACX_H
#define ACX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACX_MAX_L 128

/* call status */
#define ACX_OK 0
#define ACX_E_ARG (-1)    /* bad argument (NULL required pointer, L out of range, misaligned) */
#define ACX_E_LAUNCH (-2) /* hipLaunchKernel / hipGetLastError failed */

/* per-env error codes (err[] bytes) */
#define ACX_ERR_NONE 0
#define ACX_ERR_INVALID 1    /* reference AssertionError: invalid presentation after the move
                                (a relator became empty), utils.py:264-266 */
#define ACX_ERR_EMPTY_CONJ 2 /* reference IndexError: conjugating an empty relator,
                                ac_moves.py:117-120 */
#define ACX_ERR_DOMAIN 3     /* input outside the kernel domain: a letter not in {-2..2} or a
                                zero inside a relator (ACEnvConfig rejects both, ac_env.py:34) */
#define ACX_ERR_ACTION 4     /* move id not in [0,12) (reference AssertionError ac_moves.py:188) */

/*
 * Batched ACEnv.step / ACMove.
 *   state_in, state_out : (B,2L) int32; may alias (in place).
 *   action              : (B) int32 move ids in [0,12).
 *   reset_state         : (B,2L) int32 or NULL.  When non-NULL, an env whose step is done
 *                         or truncated is reset to its row (same-step autoreset: state_out
 *                         holds the reset state, step_count restarts at 0).
 *   step_count          : (B) int32 in/out or NULL.  Incremented per step;
 *                         truncated = step_count >= horizon (ac_env.py:102-103).
 *   reward              : (B) int32 or NULL: done ? horizon*L*2 : -(n0+n1) (ac_env.py:76,100).
 *   done, truncated     : (B) uint8 or NULL.  done = strict triviality (ac_env.py:99).
 *   lengths_out         : (B,2) int32 or NULL: relator lengths of state_out.
 *   final_obs           : (B,2L) int32 or NULL: for envs that reset, the pre-reset state
 *                         (gymnasium info["final_observation"]); other rows untouched.
 *   err                 : (B) uint8 or NULL; err_count: one int32 or NULL.
 *   cyclical            : ACEnv uses 1 (ac_env.py:93-95); greedy/bfs default 0.
 */
int acx_step(const int32_t* state_in, int32_t* state_out, const int32_t* action,
             const int32_t* reset_state, int32_t* step_count, int32_t* reward, uint8_t* done,
             uint8_t* truncated, int32_t* lengths_out, int32_t* final_obs, uint8_t* err,
             int32_t* err_count, int64_t B, int32_t L, int32_t horizon, int32_t cyclical,
             void* stream);

/*
 * T fused env steps (PPO rollout collection).  state (B,2L) and step_count (B) are
 * updated in place; actions is (T,B) int32.  Per step t the kernel writes (all optional):
 *   obs_traj[t]    (T,B,2L) int32  observation after step t (post autoreset)
 *   reward_traj[t] (T,B) int32, done_traj[t], trunc_traj[t] (T,B) uint8.
 * reset_state (B,2L) is required (autoreset on done/truncated, as acx_step).
 */
int acx_rollout(int32_t* state, const int32_t* actions, const int32_t* reset_state,
                int32_t* step_count, int32_t* obs_traj, int32_t* reward_traj, uint8_t* done_traj,
                uint8_t* trunc_traj, uint8_t* err, int32_t* err_count, int32_t T, int64_t B,
                int32_t L, int32_t horizon, int32_t cyclical, void* stream);

/*
 * 12-way neighbour expansion: for every parent (N,2L) and every move id a in [0,12)
 * the child ACMove(a, parent, L, cyclical) (greedy/bfs call it with cyclical=0).
 *   children   (N,12,2L) int32 or NULL
 *   child_len  (N,12,2) int32 or NULL
 *   child_key  (N,12,acx_key_words(L)) uint64 or NULL: packed child state (2 bits per
 *              letter, r0 then r1, then the two lengths) -- equal keys <=> equal states.
 *   err        (N,12) uint8 or NULL
 */
int acx_expand12(const int32_t* parents, int32_t* children, int32_t* child_len, uint64_t* child_key,
                 uint8_t* err, int32_t* err_count, int64_t N, int32_t L, int32_t cyclical,
                 void* stream);

/* simplify_presentation (free + optional cyclic reduction) of a batch, in/out may alias. */
int acx_canonicalize(const int32_t* state_in, int32_t* state_out, int32_t* lengths_out, uint8_t* err,
                     int32_t* err_count, int64_t B, int32_t L, int32_t cyclical, void* stream);

/* packed keys (M, acx_key_words(L)) -> presentations (M,2L) int32 (+ lengths (M,2), nullable) */
int acx_unpack_keys(const uint64_t* keys, int32_t* states, int32_t* lengths_out, int64_t M, int32_t L,
                    void* stream);

/* number of uint64 words in one packed key: ceil((4L + 16) / 64) */
int32_t acx_key_words(int32_t L);

/* library version string */
const char* acx_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ACX_H */
