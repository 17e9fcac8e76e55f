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
 *                   (ac_solver/search/greedy.py:76-83, breadth_first.py:69-76).
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
 *   - Env-step error contract (acx_step, acx_step_record, acx_step_learner and every rollout
 *     entry point; T rollout steps = T acx_step calls, tests/test_gpu_rollout_errors.py):
 *       * a failed move (ACX_ERR_INVALID, _EMPTY_CONJ, _ACTION) leaves the env's state and
 *         step count as they are for that step -- the reference raises before
 *         `count_steps += 1` (ac_env.py:93-103) -- with done = truncated = 0 and
 *         reward = -(n0+n1) of the unchanged state; the env goes on with its next move id;
 *       * a row outside the packed domain (ACX_ERR_DOMAIN) never moves and never counts; it
 *         is stored and observed with its exact int32 values.  An autoreset to such a starting
 *         row (same-step autoreset below) still happens, as the reference's reset takes any
 *         row (ac_env.py:113-129): the step reports the move's reward / done / truncated /
 *         final_obs, the env then holds that starting row with step count 0 and err
 *         ACX_ERR_DOMAIN, and lengths_out has its non-zero counts;
 *       * a rollout's err[b] is the first error of env b in the launch.
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
#define ACX_ERR_DOMAIN 3     /* input outside the packed kernels' domain: a letter not in {-2..2}
                                or a zero inside a relator.  The reference's word functions take
                                any integer letters (ACEnvConfig validates only the zero padding,
                                utils.py:13-54): the acx_word_* / acx_concatenate / acx_conjugate
                                entry points below compute those rows exactly */
#define ACX_ERR_ACTION 4     /* move id not in [0,12) (reference AssertionError ac_moves.py:188) */
#define ACX_ERR_PAD 9        /* reference ValueError: np.pad with a negative width (a relator
                                array longer than max_relator_length, utils.py:235-236) */

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
 * acx_step in place, carrying the rows' relator lengths as ACEnv does (self.lengths, set at reset
 * and passed through ACMove every step, ac_env.py:81-95,119; ac_moves.py:159,184,231): lengths (B,2) int32, in/out, holds each row's relator lengths on
 * entry and its new lengths on exit, so the kernel reads only the 16-byte chunks inside each
 * relator's letters and writes only those inside its old or new letters (the padding past both
 * already holds zeros).  Rows must be canonical (letters, then zero padding) with exact lengths;
 * (L, L) is always safe and means "read the whole row" (the next call writes the exact lengths).
 * An out-of-domain row (ACX_ERR_DOMAIN) gets (L, L).  Other arguments as acx_step; lengths is
 * required.
 */
int acx_step_lengths(int32_t* state, const int32_t* action, const int32_t* reset_state, int32_t* step_count,
                     int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths, int32_t* final_obs,
                     uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon, int32_t cyclical,
                     void* stream);

/*
 * acx_step_lengths plus a per-env reduced flag, reduced (B) uint8 in/out (required): bit 0 = both
 * relators non-empty and freely reduced, bit 1 = and cyclically reduced, as the previous call left
 * the row; 0 = unknown.  Every call writes it (a moved row: 3 when cyclical, else 1; a failed,
 * reset or out-of-domain row: 0).  A conjugation (move ids 4..11, ac_moves.py:79-156) changes only
 * its target relator, and simplify_presentation (utils.py:246-283) leaves a reduced relator as it
 * is, so for a row whose flag holds for this call's mode the relator the move leaves alone is not
 * read at all (its length is taken from `lengths`) -- except a one-letter relator (the triviality
 * test reads it) and on a step that truncates (final_obs holds the whole row).  Results are
 * acx_step's.  A caller that changes rows by other means zeroes their flags (as it resets their
 * lengths to the rows' extents).  Replaces the same reference calls as acx_step_lengths
 * (ACEnv.step -> ACMove, ac_env.py:91-111).
 */
int acx_step_lengths_reduced(int32_t* state, const int32_t* action, const int32_t* reset_state, int32_t* step_count,
                             int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths, uint8_t* reduced,
                             int32_t* final_obs, uint8_t* err, int32_t* err_count, int64_t B, int32_t L,
                             int32_t horizon, int32_t cyclical, void* stream);

/*
 * A per-call step plan: acx_step, acx_step_lengths or acx_step_lengths_reduced (kind
 * ACX_STEP_PLAN_STEP / _LENGTHS / _LENGTHS_REDUCED) with every argument but the move ids and the
 * stream resolved once, for a caller that steps the same buffers every call (BASELINE configs[1]:
 * 65,536 envs stepped 200 times; ACEnv.step per call, ac_env.py:91-111).  acx_step_plan_create
 * takes that entry's arguments (state_out == state_in and lengths required for the lengths kinds,
 * reduced only and required for _LENGTHS_REDUCED) and makes its argument checks once; it returns
 * NULL when they fail or memory is short.  acx_step_plan_launch(plan, action, stream) is then that
 * entry with those arguments -- same kernels, results and return codes (ACX_E_ARG for a NULL
 * plan).  The plan holds the pointers, not the buffers: they must outlive it.  The plan is host
 * memory; launches from several threads may share one plan, destroy it once (NULL is a no-op).
 */
typedef struct acx_step_plan acx_step_plan;
#define ACX_STEP_PLAN_STEP 0
#define ACX_STEP_PLAN_LENGTHS 1
#define ACX_STEP_PLAN_LENGTHS_REDUCED 2
acx_step_plan* acx_step_plan_create(int32_t kind, const int32_t* state_in, int32_t* state_out,
                                    const int32_t* reset_state, int32_t* step_count, int32_t* reward, uint8_t* done,
                                    uint8_t* truncated, int32_t* lengths, uint8_t* reduced, int32_t* final_obs,
                                    uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
                                    int32_t cyclical);
int acx_step_plan_launch(const acx_step_plan* plan, const int32_t* action, void* stream);
void acx_step_plan_destroy(acx_step_plan* plan);

/*
 * acx_step for the PPO learner (ac_solver/agents/training.py:221-356), state updated in place
 * with same-step autoreset to reset_state, plus the learner-side writes fused in:
 *   action / action_i64 : exactly one non-NULL; action_i64 = the policy's int64 samples
 *                         (training.py:232-236), out of [0,12) -> ACX_ERR_ACTION.
 *   obs_f32     (B,2L) float32 or NULL: the next observation (post reset), written straight
 *               into the learner's buffer (e.g. obs[t+1], training.py:151-153,225).
 *   reward_f32  (B) float32 or NULL (rewards[t], training.py:241-253).
 *   done_f32    (B) float32 or NULL: done only, as next_done = torch.Tensor(done) (:354-356).
 *   done, truncated (B) uint8 or NULL.
 *   action_hist (hist_cap, B) uint8 or NULL: the moves of each env's current episode
 *               (ACEnv.actions / info["actions"], ac_env.py:96,105; training.py:275-280),
 *               step-major: with hist_base NULL move k of env i is at [k, i]; with hist_base
 *               ((B) int32, in/out) it is at [(hist_base[i] + k) mod hist_cap, i] and an
 *               episode's move 0 sets hist_base[i] = hist_t mod hist_cap -- hist_t is the
 *               caller's step counter (+1 per call) -- so every env writes this step's move to one
 *               row, coalesced, however far apart the envs' episodes are.  Read an ended
 *               episode's moves right after its last step (the next call may start the ring
 *               over them); an episode longer than hist_cap moves keeps its first hist_cap.
 *   episode_len (B) int32 or NULL: the length of the episode that ended this step, else 0.
 *   step_count is required (truncation, history position).
 */
int acx_step_learner(int32_t* state, const int32_t* action, const int64_t* action_i64, const int32_t* reset_state,
                     int32_t* step_count, float* obs_f32, float* reward_f32, float* done_f32, uint8_t* done,
                     uint8_t* truncated, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                     int32_t* episode_len, int32_t* final_obs, uint8_t* err, int32_t* err_count, int64_t B, int32_t L,
                     int32_t horizon, int32_t cyclical, void* stream);

/*
 * acx_step plus the episode move history gymnasium's SyncVectorEnv hands the trainer
 * (ac_env.py:92,105-110 -> infos["final_info"][i]["actions"] / infos["actions"][i],
 * training.py:273-280): action_hist (hist_cap, B) uint8 and hist_base / hist_t as
 * acx_step_learner; episode_len (B) int32 or NULL = the length of the episode that ended this step
 * (done | truncated), else 0.  step_count and action_hist are required; other arguments as
 * acx_step.
 */
int acx_step_record(const int32_t* state_in, int32_t* state_out, const int32_t* action, const int32_t* reset_state,
                    int32_t* step_count, int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths_out,
                    int32_t* final_obs, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                    int32_t* episode_len, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
                    int32_t cyclical, void* stream);

/*
 * acx_step with gymnasium >= 1.0's NEXT_STEP autoreset instead of the same-step one (the
 * reference trainer reads either info layout, training.py:273-280; gymnasium is an
 * un-vendored dependency, so this timing is parity unpinned).  pending (B) uint8, in/out: an
 * env whose flag is set is reset to its reset_state row on this call instead of stepping --
 * its action is ignored, reward 0, done = truncated = 0, step count 0 -- and every env's flag
 * becomes done | truncated of this call, so the step that ends an episode returns the terminal
 * state itself.  action_hist / hist_cap / hist_base / hist_t / episode_len: as acx_step_record
 * (NULL / 0 / NULL / 0 / NULL for none).  reset_state and step_count are required; other arguments as acx_step (no final_obs:
 * the ending step's state is the observation).
 */
int acx_step_next(const int32_t* state_in, int32_t* state_out, const int32_t* action, const int32_t* reset_state,
                  int32_t* step_count, int32_t* reward, uint8_t* done, uint8_t* truncated, int32_t* lengths_out,
                  uint8_t* pending, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                  int32_t* episode_len, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t horizon,
                  int32_t cyclical, void* stream);

/*
 * Start-state curriculum of the PPO trainer, round 1 (training.py:319-352): every env whose
 * episode ended this step (done | truncated), in env order, starts next from
 * curriculum_states[k], k = *next_index, *next_index + 1, ... (max(states_processed) + 1);
 * its state, reset_state (nullable) and obs_f32 (nullable) rows are set to that state and
 * curr_index[env] = k.  When k reaches n_states round 1 is complete and the env is flagged in
 * needs_host[env] = 1 (the reference then draws a random solved/unsolved state on the host).
 * workspace: acx_curriculum_workspace(B) int32 device words, 8-byte aligned, zeroed before the
 * first call and not written by the caller afterwards (acx_learner_step keeps its look-back state
 * there; one workspace serves both calls; concurrent launches on one workspace are unsupported --
 * their results are undefined and nothing detects them).  For even L the row
 * arrays (curriculum_states, state, reset_state, obs_f32) are 16-byte aligned.
 */
int64_t acx_curriculum_workspace(int64_t B);
int acx_curriculum_assign(const uint8_t* done, const uint8_t* truncated, const int32_t* curriculum_states,
                          int64_t n_states, int32_t* next_index, int32_t* curr_index, uint8_t* needs_host,
                          int32_t* state, int32_t* reset_state, float* obs_f32, int32_t* workspace, int64_t B,
                          int32_t L, void* stream);

/*
 * One PPO env step = acx_step_learner (final_obs NULL) followed by acx_curriculum_assign
 * (training.py:238-241, 319-352), in ONE launch with the same results: the step kernel ranks the
 * finished envs in env order itself (per-64-env-tile counts and per-group totals in the
 * workspace) and, after a tile's own stores, a finished env with index k < n_states takes initial
 * state k -- its state, obs_f32 and reset_state rows become that row as it is, curr_index[env] = k;
 * past the table's end needs_host[env] = 1.  When the table surely lasts the launch
 * (*next_index + B <= n_states) a finished env is not autoreset first: its rows are written once,
 * from the curriculum row, and its err reports the step alone (acx_step_learner's autoreset would
 * add err 3 for an out-of-domain reset_state row; LearnerEnv's rows never differ that way: an env
 * holding an out-of-domain row fails every step and never finishes).
 * needs_host[env] = 3: the ranking gave up (an earlier
 * tile not scheduled within ~seconds); the env kept its own starting row and was not ranked.  Any
 * give-up -- a tile's ranking, or the last tile's total, after which *next_index is stale -- also
 * sets the workspace's sticky failure word (acx_learner_failure_word); from then on every launch
 * ranks nothing (finished envs: needs_host 3) until the caller re-zeroes the workspace and
 * restores *next_index (max(curr_index) + 1 in round 1: every finished env that was ranked holds
 * its state).  done, truncated, reset_state and the curriculum arguments are required; B < 2^31;
 * workspace = acx_curriculum_workspace(B) int32 words (above); for even L, reset_state and
 * curriculum_states 16-byte aligned (as state and obs_f32).
 */
int acx_learner_step(int32_t* state, const int32_t* action, const int64_t* action_i64, int32_t* reset_state,
                     int32_t* step_count, float* obs_f32, float* reward_f32, float* done_f32, uint8_t* done,
                     uint8_t* truncated, uint8_t* action_hist, int32_t hist_cap, int32_t* hist_base, int64_t hist_t,
                     int32_t* episode_len, uint8_t* err, int32_t* err_count, const int32_t* curriculum_states,
                     int64_t n_states, int32_t* next_index, int32_t* curr_index, uint8_t* needs_host,
                     int32_t* workspace, int64_t B, int32_t L, int32_t horizon, int32_t cyclical, void* stream);
/* the int32 index, in a workspace of acx_curriculum_workspace(B) words, of acx_learner_step's
 * sticky failure word (a uint64: 0 while every ranking has completed) */
int64_t acx_learner_failure_word(int64_t B);

/*
 * T fused env steps (PPO rollout collection).  state (B,2L) and step_count (B) are
 * updated in place; actions is (T,B) int32.  Per step t the kernel writes (all optional):
 *   obs_traj[t]    (T,B,2L) int32  observation after step t (post autoreset)
 *   reward_traj[t] (T,B) int32, done_traj[t], trunc_traj[t] (T,B) uint8.
 * reset_state (B,2L) is required (autoreset on done/truncated, as acx_step).  Errors follow the
 * env-step error contract above, so the trajectory equals T acx_step calls; err[b] is env b's
 * first error in the launch.
 */
int acx_rollout(int32_t* state, const int32_t* actions, const int32_t* reset_state,
                int32_t* step_count, int32_t* obs_traj, int32_t* reward_traj, uint8_t* done_traj,
                uint8_t* trunc_traj, uint8_t* err, int32_t* err_count, int32_t T, int64_t B,
                int32_t L, int32_t horizon, int32_t cyclical, void* stream);

/*
 * The same rollout with the move ids pre-packed by acx_pack_actions: packed_actions is
 * (ceil(T/8), B) uint32, word [t/8][i] holding the ids of env i at steps 8(t/8)..+7, 4 bits
 * each (an id outside [0,12) as 15).  acx_pack_actions + acx_rollout_packed give the same
 * results as acx_rollout; the rollout then reads 0.5 B of ids per env-step instead of 4
 * (scattered id reads between the trajectory write bursts are what costs).
 * acx_packed_actions_words(T, B) = number of uint32 words of packed_actions.
 */
int64_t acx_packed_actions_words(int32_t T, int64_t B);
int acx_pack_actions(const int32_t* actions, uint32_t* packed_actions, int32_t T, int64_t B, void* stream);
int acx_rollout_packed(int32_t* state, const uint32_t* packed_actions, const int32_t* reset_state,
                       int32_t* step_count, int32_t* obs_traj, int32_t* reward_traj, uint8_t* done_traj,
                       uint8_t* trunc_traj, uint8_t* err, int32_t* err_count, int32_t T, int64_t B,
                       int32_t L, int32_t horizon, int32_t cyclical, void* stream);

/*
 * The rollout with the observation trajectory as int8 letters, obs_traj8 (T,B,2L) int8: the
 * dtype of the reference's observation_space (ac_env.py:64-70, Box(int8)) and of the
 * observations gymnasium's SyncVectorEnv returns (environment.py:70-72), a quarter of the
 * int32 trajectory's bytes.  Exactly one of actions ((T,B) int32) / packed_actions
 * (acx_pack_actions) is given; everything else as acx_rollout.
 */
int acx_rollout_obs8(int32_t* state, const int32_t* actions, const uint32_t* packed_actions,
                     const int32_t* reset_state, int32_t* step_count, int8_t* obs_traj8, int32_t* reward_traj,
                     uint8_t* done_traj, uint8_t* trunc_traj, uint8_t* err, int32_t* err_count, int32_t T,
                     int64_t B, int32_t L, int32_t horizon, int32_t cyclical, void* stream);

/*
 * 12-way neighbour expansion: for every parent (N,2L) and every move id a in [0,12)
 * the child ACMove(a, parent, L, cyclical) (greedy/bfs call it with cyclical=0).
 *   children   (N,12,2L) int32 or NULL
 *   child_len  (N,12,2) int32 or NULL
 *   child_key  (N,12,acx_key_words(L)) uint64 or NULL: packed child state (2 bits per
 *              letter, r0 then r1, then the two lengths) -- equal keys <=> equal states.
 *              The key of a child whose move failed (err != 0) has both length bytes
 *              0xFF, which no state has.
 *   err        (N,12) uint8 or NULL
 */
int acx_expand12(const int32_t* parents, int32_t* children, int32_t* child_len, uint64_t* child_key,
                 uint8_t* err, int32_t* err_count, int64_t N, int32_t L, int32_t cyclical,
                 void* stream);

/* simplify_presentation (free + optional cyclic reduction) of a batch, in/out may alias. */
int acx_canonicalize(const int32_t* state_in, int32_t* state_out, int32_t* lengths_out, uint8_t* err,
                     int32_t* err_count, int64_t B, int32_t L, int32_t cyclical, void* stream);

/*
 * The reference's word functions on ARBITRARY int32 letters (csrc/acx_words.hip): exact, including
 * letters beyond +-2 (its unit tests use 3..6) and zeros inside a relator, one lane per row with
 * the rows staged through LDS.  A row whose reference call raises keeps its input and gets the
 * ACX_ERR_* code of the exception (err / err_count nullable).
 *   acx_word_move      ACMove (ac_moves.py:159-231) per row: move id action[b]; lengths_out (B,2);
 *                      done (nullable) = strict triviality of the result (ac_env.py:99)
 *   acx_concatenate    concatenate_relators (ac_moves.py:4-76): r_i <- r_i r_j^sign, no reduction;
 *                      lengths_out = the caller's lengths_in (or the non-zero counts when NULL)
 *                      with [i] replaced by the new size when it fits (the reference updates the
 *                      list it is given)
 *   acx_conjugate      conjugate (ac_moves.py:79-156): r_i <- x_j^sign r_i x_j^-sign, no reduction
 *   acx_word_simplify_presentation  simplify_presentation (utils.py:246-283)
 *   acx_word_simplify_relator  simplify_relator (utils.py:178-243) on (B, m) relator arrays: out
 *                      (B, max(m, L)) holds the returned array in its first out_len[b] entries
 *                      (L when padded), n_out[b] the word length
 */
int acx_word_move(const int32_t* state_in, int32_t* state_out, const int32_t* action, int32_t* lengths_out,
                  uint8_t* done, uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t cyclical,
                  void* stream);
int acx_concatenate(const int32_t* state_in, int32_t* state_out, const int32_t* lengths_in, int32_t* lengths_out,
                    int64_t B, int32_t L, int32_t i, int32_t j, int32_t sign, void* stream);
int acx_conjugate(const int32_t* state_in, int32_t* state_out, const int32_t* lengths_in, int32_t* lengths_out,
                  uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t i, int32_t j, int32_t sign,
                  void* stream);
int acx_word_simplify_presentation(const int32_t* state_in, int32_t* state_out, int32_t* lengths_out, uint8_t* err,
                                   int32_t* err_count, int64_t B, int32_t L, int32_t cyclical, void* stream);
int acx_word_simplify_relator(const int32_t* relators, int32_t m, int32_t* out, int32_t* out_len, int32_t* n_out,
                              uint8_t* err, int32_t* err_count, int64_t B, int32_t L, int32_t cyclical,
                              int32_t padded, void* stream);

/* packed keys (M, acx_key_words(L)) -> presentations (M,2L) int32 (+ lengths (M,2), nullable) */
int acx_unpack_keys(const uint64_t* keys, int32_t* states, int32_t* lengths_out, int64_t M, int32_t L,
                    void* stream);

/*
 * Breadth-first search entirely on the GPU (replaces bfs, ac_solver/search/breadth_first.py:15-97,
 * with identical results): FIFO queue of packed node keys and the visited set (open-addressing
 * hash table) in HBM; the 12-way expansion, dedup against the visited set and within the chunk
 * (first occurrence in (parent, action) order wins), the success test and the per-parent node
 * budget run as kernels over chunks of up to `chunk_parents` parents (<= 0: 2^20).
 *   acx_bfs_create   allocates the device workspace on the current device for searches of
 *                    up to max_nodes nodes (<= 2^30) at max_relator_length L; NULL on failure
 *                    (every child key of every expanded parent is kept: ~12 * 8 * kw bytes
 *                    per node, 2.9 GB at 10^7 nodes and L = 36).
 *   acx_bfs_run      searches from `presentation` (HOST pointer, 2L int32, a valid presentation
 *                    with letters +-1, +-2) with budget max_nodes (<= the create-time value);
 *                    synchronous on `stream`: when it returns, `stream` is idle (every chunk
 *                    it enqueued, the speculative one after the search's end included, has
 *                    retired).  A chunk that does not publish its state within 30 s (a kernel
 *                    that does not finish) returns ACX_E_LAUNCH.  On ACX_BFS_FOUND the reference's path
 *                    [(-1, initial total), (action, total)...] is written to path_actions /
 *                    path_totals (first path_cap entries).  stats (int64[5]) = n_nodes
 *                    (len(tree_nodes) at the end), parents expanded, chunks, min total length
 *                    seen, path length.  Returns an ACX_BFS_* status or a negative ACX_E_*.
 */
#define ACX_BFS_EXHAUSTED 0  /* queue ran empty: (False, None) */
#define ACX_BFS_FOUND 1      /* (True, path) */
#define ACX_BFS_BUDGET 2     /* len(tree_nodes) >= max_nodes after a parent: (False, None) */
#define ACX_BFS_MOVE_ERROR 3 /* an ACMove raised AssertionError (a relator became empty) */
void* acx_bfs_create(int32_t L, int64_t max_nodes, int64_t chunk_parents, int32_t cyclical);
int acx_bfs_run(void* h, const int32_t* presentation, int64_t max_nodes, int32_t* path_actions,
                int32_t* path_totals, int64_t path_cap, int64_t* stats, void* stream);
void acx_bfs_destroy(void* h);
/* packed keys (acx.h key format) of the first min(cap, n) nodes of the last run in discovery
   (FIFO) order, n = nodes held (<= max_nodes + 12); returns n */
int64_t acx_bfs_node_keys(void* h, uint64_t* out, int64_t cap, void* stream);
/* the new minimal total lengths of the last run in the order the reference finds them (its
   verbose "New minimal length found: m" lines, breadth_first.py:79-82): writes the first cap,
   returns how many there are */
int64_t acx_bfs_min_trace(void* h, int32_t* out, int64_t cap);

/*
 * Breadth-first search with the node store and the visited set partitioned over G GPUs by key
 * owner (one process per GPU).  Same results as acx_bfs_run / the
 * reference bfs (breadth_first.py:15-97).  The caller runs the same chunk loop on every rank
 * (acx/search/_sharded_bfs.py) and does the exchanges between the calls:
 *   acx_sbfs_create    workspace on the current device: this rank's node store (local_cap
 *                      nodes), chunks of <= chunk_parents parents (<= 0 or the maximum: 2^19);
 *                      NULL on failure.  Keys live in an arena of expanded children that
 *                      acx_sbfs_expand grows by doubling when a chunk would not fit (a failed
 *                      allocation there returns ACX_E_LAUNCH)
 *   acx_sbfs_owner     owner rank of a presentation's key (HOST pointer)
 *   acx_sbfs_reset     new search from `presentation` (HOST); returns the root's owner rank
 *   acx_sbfs_expand    expands this rank's parents among global ids [head, head + P);
 *                      read_back != 0: waits for it and writes out int64[5 + world] = success
 *                      seq, move-error seq (0xffffffff: none), min child total, local parents,
 *                      overflow, children per owner; read_back = 0 (one rank: nothing to
 *                      exchange) returns at once -- the same fields come back from the commit
 *   acx_sbfs_pack      the children other ranks own into `send` ((n, kw + 1) uint64: key
 *                      words, chunk seq), grouped by owner in rank order (the count for the
 *                      rank itself is 0: its own children are inserted in place)
 *   -- all_to_all of the records: recv holds the records every rank sent to this one --
 *   acx_sbfs_insert    probe / claim the visited set with this rank's own children and the
 *                      received records, up to seq `end` (end < 0: this rank's own first
 *                      success / move error, i.e. one rank's); survivors as bits of gmask ((P)
 *                      uint32, written by the call -- or, with end < 0 at one rank, where
 *                      nothing is exchanged, by the acx_sbfs_commit that follows)
 *   -- all_reduce (sum) of gmask over the ranks --
 *   acx_sbfs_commit    global ids, the node-budget cut and the appends; out int64[9] = nodes
 *                      appended (all ranks), cut parent (-1: none), nodes after the cut
 *                      parent, nodes appended here, overflow flags, then this rank's expansion
 *                      of the chunk: success seq, move-error seq, min child total, local parents
 *   acx_sbfs_min_len   min child total over this rank's parents of the last chunk up to `last`
 *   acx_sbfs_lookup    out int64[4] = found, parent id, action, total of the node with id g
 *   acx_sbfs_node_keys this rank's nodes (keys, global ids; ascending id); returns the count
 *   acx_sbfs_max_records  capacity of send / recv in records (12 * chunk_parents)
 * All calls are on `stream`; expand, commit, min_len, lookup and reset synchronise it.
 */
void* acx_sbfs_create(int32_t L, int64_t local_cap, int64_t chunk_parents, int32_t cyclical, int32_t rank,
                      int32_t world);
void acx_sbfs_destroy(void* h);
int64_t acx_sbfs_max_records(void* h);
int32_t acx_sbfs_owner(const int32_t* presentation, int32_t L, int32_t world);
int acx_sbfs_reset(void* h, const int32_t* presentation, void* stream);
int acx_sbfs_expand(void* h, int64_t head, int32_t P, int64_t* out, int32_t read_back, void* stream);
int acx_sbfs_pack(void* h, uint64_t* send, void* stream);
int acx_sbfs_insert(void* h, const uint64_t* recv, int64_t nrecv, int64_t end, uint32_t* gmask, void* stream);
int acx_sbfs_commit(void* h, const uint32_t* gmask, int64_t n_before, int64_t need, int64_t* out, void* stream);
int64_t acx_sbfs_min_len(void* h, int64_t last, void* stream);
int acx_sbfs_lookup(void* h, int64_t g, int64_t* out, void* stream);
/* verbose trace of the last chunk (after acx_sbfs_commit; breadth_first.py:79-82): this rank's
 * children with seq < end whose total is below `running` and below every earlier child of this
 * rank, as (seq, total) int64 pairs into out (HOST, 2 * cap); returns their count.  The caller
 * merges every rank's records in seq order to print the reference's new-minimum lines. */
int64_t acx_sbfs_trace(void* h, int64_t running, int64_t end, int64_t* out, int64_t cap, void* stream);
int64_t acx_sbfs_node_keys(void* h, uint64_t* keys, int64_t* gids, int64_t cap, void* stream);

/*
 * Scoring inputs for value-guided search (value_search/): exactly one of `states` ((M,2L) int32)
 * or `keys` ((M, acx_key_words(L)) packed keys, e.g. acx_expand12 output) is non-NULL.
 *   acx_features   out (M,14) float32 = compute_features (feature_extraction.py:11-91); with
 *                  mean/std (14 float32 each, both or neither) normalised (f - mean) / std as
 *                  _score_states_mlp does (value_guided_search.py:49-66).
 *   acx_token_ids  out (M, max_state_dim) int64 = letter + 2, padded with 2
 *                  (_score_states_seq, value_guided_search.py:68-84); max_state_dim >= 2L.
 */
int acx_features(const int32_t* states, const uint64_t* keys, const float* mean, const float* stdv, float* out,
                 int64_t M, int32_t L, void* stream);
int acx_token_ids(const int32_t* states, const uint64_t* keys, int64_t* out, int64_t M, int32_t L,
                  int32_t max_state_dim, void* stream);

/*
 * Host search engine (csrc/acx_search.cpp) for greedy_search (greedy.py:15-121) and bfs with
 * host-side dedup: the caller expands the parents the engine asks for with acx_expand12
 * (packed keys) and feeds the child keys back; the engine replays the reference's pop /
 * expand / dedup / budget order exactly.  mode 0 = bfs, 1 = greedy.
 *   acx_search_next_batch  up to cap parent keys to expand next (0: nothing left)
 *   acx_search_feed        the (count, 12, kw) child keys of the last batch; returns status
 *   acx_search_status      0 running, 1 success, 2 failed, 3 a child move raised (its key
 *                          is the acx_expand12 error sentinel): the reference's AssertionError
 *   acx_search_path        the result path (see acx_search.cpp); returns its length
 *   acx_search_stats       out[0] rounds, out[1] parents expanded, out[2] parents popped,
 *                          out[3..5] host ns in next_batch / caching children / the replay
 *   acx_search_node_keys   the packed keys of the discovered nodes in discovery order
 *   acx_search_min_trace   the new minimum totals in the order found (the verbose "New minimal
 *                          length found" lines, greedy.py:86-89, breadth_first.py:79-82)
 *   acx_search_popped      the ids (discovery index) of the expanded nodes in pop order
 *   acx_search_found       after a success: the first letters of the found child's relators and
 *                          len(tree_nodes) - len(to_explore) then (greedy.py:92-95); returns 1
 */
void* acx_search_create(int32_t mode, int32_t L, const uint64_t* start_key, int64_t max_nodes);
void acx_search_destroy(void* h);
int64_t acx_search_next_batch(void* h, uint64_t* parent_keys, int64_t cap);
int32_t acx_search_feed(void* h, const uint64_t* child_keys, int64_t count);
int32_t acx_search_status(void* h, int32_t* budget_hit, int32_t* min_length, int64_t* n_nodes);
int64_t acx_search_path(void* h, int32_t* actions, int32_t* totals, int64_t cap);
void acx_search_stats(void* h, int64_t* out);
int64_t acx_search_node_keys(void* h, uint64_t* out, int64_t cap);
int64_t acx_search_min_trace(void* h, int32_t* out, int64_t cap);
int64_t acx_search_popped(void* h, int64_t* ids, int64_t cap);
int32_t acx_search_found(void* h, int32_t* first_letters, int64_t* explored);

/*
 * greedy_search (greedy.py:15-121) with the visited set on the device (csrc/acx_greedy.hip): the
 * expansion rounds are driven from C++ on the current device -- each round expands the smallest
 * frontier nodes not yet expanded (lane per (parent, action)) and probes every child against the
 * HBM hash table of the committed nodes; the host replays the reference's pop / dedup / budget
 * order exactly, checking only the children the device did not know against the nodes appended
 * since (the in-flight conflicts).  batch = parents per round (<= 0: 64).
 *   acx_greedy_run       searches from `presentation` (HOST pointer, 2L int32, letters +-1/+-2),
 *                        max_nodes <= 2^38; the device key store and visited set start at
 *                        min(max_nodes, 2^22) nodes and double as the search grows;
 *                        *out_handle receives the finished search (query it, then destroy)
 *   acx_greedy_status / _path / _min_trace / _popped / _node_keys / _found   as acx_search_*
 *   acx_greedy_stats     out[0] rounds, [1] parents expanded, [2] popped, [3] children the device
 *                        knew, [4..6] host ns selecting / GPU round trips / replaying, [7..9] replays
 *                        stopped at a node appended in that replay / an older unexpanded node / an
 *                        aged cache, [10..11] ns of the round trips spent polling for the GPU /
 *                        caching children, [12] cached expansions retired unused because they aged
 *                        (13 int64)
 */
int acx_greedy_run(const int32_t* presentation, int32_t L, int64_t max_nodes, int32_t cyclical, int32_t batch,
                   void** out_handle);
void acx_greedy_destroy(void* h);
int32_t acx_greedy_status(void* h, int32_t* budget_hit, int32_t* min_length, int64_t* n_nodes);
int64_t acx_greedy_path(void* h, int32_t* actions, int32_t* totals, int64_t cap);
void acx_greedy_stats(void* h, int64_t* out);
int64_t acx_greedy_min_trace(void* h, int32_t* out, int64_t cap);
int64_t acx_greedy_popped(void* h, int64_t* ids, int64_t cap);
int64_t acx_greedy_node_keys(void* h, uint64_t* out, int64_t cap);
int32_t acx_greedy_found(void* h, int32_t* first_letters, int64_t* explored);

/* number of uint64 words in one packed key: ceil((4L + 16) / 64) */
int32_t acx_key_words(int32_t L);

/* library version string */
const char* acx_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ACX_H */
