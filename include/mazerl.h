/* mazerl.h — C ABI of libmazerl.so, the MI355X-native batched maze environment.
 *
 * The reference (Fabri000/Maze-Solving-Agent-Gymnasium) has no FFI: its boundary is the Python
 * gym.Env class API. This header is the drop-in boundary underneath that API:
 * the Python classes in maze-solving-agent-gymnasium_amd/mazerl/ bind these entry points with
 * ctypes (INTEGRATION.md shows the binding). Each entry point names the reference interface it
 * replaces (file:line in the reference).
 *
 * Conventions
 *   - Every call returns an int status: MZ_OK (0) or a negative MZ_E* code; mz_last_error()
 *     returns the thread-local message of the last failure.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream). Calls are async on it
 *     unless documented as synchronous.
 *   - Pointers named *_dev are device (HBM) pointers owned by the caller (e.g. torch tensors);
 *     pointers named *_host are host pointers. The handle owns all per-instance env state.
 *   - One handle per stream/thread; handles are not internally locked. Instances (envs) of a
 *     handle are fully independent (no global mutable state, per-instance algorithm id).
 *   - Grids are uint8, row-major, 0 = wall, 1 = floor, 2 = goal (lib/maze_generation.py:16).
 *     Shapes must be square and odd (the reference raises IndexError for even N),
 *     5 <= N <= MZ_MAX_DIM. Window (enrich) mode needs N >= 15 for euclidean mazes (Q7).
 */
#ifndef MAZERL_H
#define MAZERL_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MZ_OK 0
#define MZ_EINVAL (-1)       /* bad argument */
#define MZ_EINVAL_SHAPE (-2) /* grid shape the reference cannot represent (even N, N<15 window) */
#define MZ_EHIP (-3)         /* HIP runtime error */
#define MZ_ENOMEM (-4)
#define MZ_EALIGN (-5)       /* output pointer misaligned (window f32 needs 16 B) */

#define MZ_MAX_DIM 127
#define MZ_BANK_MAX_DIMS 64  /* maze sizes one bank can hold (mz_bank_create_dims) */
#define MZ_MAX_CANDIDATES 64 /* candidates of a best-of-C selection (mz_bank_create_ex, mz_generate_best) */
#define MZ_WINDOW 15
#define MZ_WINDOW_BITS 675   /* 3 x 15 x 15 */
#define MZ_WINDOW_WORDS 22   /* uint32 words per instance in window_bits (bits 675..703 zero) */

/* algorithm ids (BaseMazeEnv.ALGORITHM strings, base_maze_env.py:17; maze_generation.py:24-30) */
#define MZ_ALGO_RPRIM 0
#define MZ_ALGO_DFS 1
#define MZ_ALGO_PRIMKILL 2

typedef struct mz_handle mz_handle;

typedef struct {
  int32_t num_envs;  /* B: independent env instances on this GPU */
  int32_t max_dim;   /* storage pitch: every instance's N <= max_dim */
  int32_t toroidal;  /* 0 euclidean (SimpleMazeEnv family), 1 toroidal (ToroidalMazeEnv family) */
  int32_t enrich;    /* 1 = *Enrich* observation (3x15x15 window), 0 = plain obs */
  int32_t device;    /* HIP device ordinal */
  int32_t reserved[7];
} mz_config;

/* Per-step outputs; every pointer is a caller-owned device buffer and may be NULL (= not
 * written). Reward dtype note: the reference returns Python floats/ints; reward64 carries the
 * exact value, reward is its float32 rounding (what torch.tensor(batch.reward) holds). */
typedef struct {
  float* reward;          /* [B] */
  double* reward64;       /* [B] */
  uint8_t* terminated;    /* [B] */
  uint8_t* truncated;     /* [B] */
  int32_t* pos;           /* [B][2] agent (row, col)           obs["agent"] (plain) */
  int32_t* best_dir;      /* [B][2] agent - best_next_cell     obs["best dir"] */
  float* obs6;            /* [B][6] learner state vector concat(agent, target, best dir) as f32,
                             enrich: agent/maze_shape, target/maze_shape (off_policy_trainer.py:156) */
  uint32_t* window_bits;  /* [B][22] 675-bit 3x15x15 window, channel-major, LSB-first */
  float* window;          /* [B][3][15][15] f32 obs["window"] (get_mask_tensor), 16 B aligned */
  int32_t* done_idx;      /* [B] indices of instances whose step ended terminated|truncated */
  int32_t* done_count;    /* [1] number of valid done_idx entries (caller zeroes it first) */
} mz_step_out;

typedef struct { /* host-side snapshot of one instance (mz_query) */
  int32_t n, start_r, start_c, goal_r, goal_c, max_steps;
  int32_t r, c, steps, invalid_streak, nmoves, last_action, done;
} mz_env_info;

const char* mz_last_error(void);
int mz_device_count(int* n);

/* Create / destroy a batch of B env instances on one GPU. */
int mz_create(const mz_config* cfg, mz_handle** out);
int mz_destroy(mz_handle* h);

/* Import mazes bit-exactly (e.g. reference-generated fixtures) into instances env_ids_host[i]
 * (NULL = 0..n-1). grids_host is [n][dim][dim]; start_goal_host is [n][4] (sr, sc, gr, gc).
 * Builds the per-maze distance field / move tables, max_steps, and resets the instances.
 * Replaces: env construction with a given maze (SimpleMazeEnv.__init__, simple_maze_env.py:19-36)
 * and set_max_steps (:52-58). Synchronous. */
int mz_load_mazes(mz_handle* h, const uint8_t* grids_host, int32_t dim,
                  const int32_t* start_goal_host, const int32_t* env_ids_host, int32_t n,
                  void* stream);

/* Generate new mazes on the GPU for the listed instances (env_ids_dev NULL = all B) with the
 * per-instance algorithm ids (algo_dev [n] or NULL = algo_all) and Philox seeds
 * seed + env_id; then builds tables and resets them. Replaces gen_maze / gen_maze_no_border
 * (maze_generation.py:6-56) + update_new_maze (simple_maze_env.py:118-127) with candidates=1
 * (the best-of-6 difficulty selection, base_maze_env.py:78-97, is mz_generate_best). */
int mz_generate(mz_handle* h, const int32_t* env_ids_dev, int32_t n, const uint8_t* algo_dev,
                int32_t algo_all, int32_t dim, uint64_t seed, void* stream);

/* Best-of-C generation: the reference's new-maze selection (BaseMazeEnv.generate_maze,
 * base_maze_env.py:78-97; ToroidalMazeEnv.generate_maze, toroidal_maze_env.py:40-54: six
 * gen_maze / gen_maze_no_border candidates, the one with the smallest McClendon difficulty —
 * maze_complexity_evaluation.py:319-329, a toroidal maze scored as its bordered maze — kept, the
 * first on ties) for the listed instances, on the GPU: `candidates` Philox mazes per instance
 * (candidate c of instance e: seed + e * candidates + c, the mazes mz_generate of
 * n * candidates instances from `seed` builds for instances e * candidates + c), scored by the
 * difficulty kernel, the first minimum copied into the instance (which is then reset like after
 * mz_generate). Euclidean handles score every candidate first with the order-free screen
 * (mz_screen_batch) and decide a group from it when its minimum is separated from every other
 * candidate by more than the screen's rigorous error bounds (+ 2^-40); the other groups are
 * rebuilt and scored by the order-exact kernel (mz_difficulty_batch), and a candidate that kernel
 * declines is scored by the host restatement (mz_difficulty) inside the stream
 * (hipLaunchHostFunc), so every candidate of a group is compared. candidates == 1 is
 * mz_generate_ex(MZ_RNG_PHILOX). Selection statistics:
 * mz_select_stats. Replaces update_new_maze (simple_maze_env.py:118-127) / the env constructors'
 * first maze (simple_maze_env.py:19-36). */
int mz_generate_best(mz_handle* h, const int32_t* env_ids_dev, int32_t n, const uint8_t* algo_dev,
                     int32_t algo_all, int32_t dim, uint64_t seed, int32_t candidates,
                     void* stream);
/* Counters of every best-of-C selection on this handle (bank refills and mz_generate_best) ->
 * out3_dev [3] int32 (device, nullable): groups with a candidate the GPU difficulty kernel leaves
 * to the host (status != 0; the group picks among the others), groups where a candidate listed
 * before the chosen one lies within a relative 2^-40 of its difficulty product (its log could
 * tie the chosen one's: the reference would keep the earlier), groups selected. reset != 0 zeroes
 * them after the copy. */
int mz_select_stats(mz_handle* h, int32_t* out3_dev, int32_t reset, void* stream);
/* The same counters, the first n (<= MZ_SELECT_STATS) of: [0] unresolved groups (a candidate
 * with no score from the GPU kernels or the host — or a group past the exact path's per-run cap
 * of 256, which keeps the screen's pick), [1] near ties (as above), [2] groups selected, [3]
 * groups the screen left to the order-exact kernel, [4] candidates scored by the host
 * restatement. */
#define MZ_SELECT_STATS 5
int mz_select_stats_ex(mz_handle* h, int32_t* out_dev, int32_t n, int32_t reset, void* stream);
/* Test hooks of the best-of-C pipeline (flags, 0 = off): 1 every group to the order-exact
 * kernel, 2 even-numbered candidates treated as declined by it (host-scored), 4 all candidates of
 * a group from one seed (exact ties). */
int mz_set_debug(mz_handle* h, int32_t flags);
/* Per-instance size of a winner's next maze for mz_reset_done / mz_reset_list with regen_won:
 * dims_dev [B] uint8 (device, owned by the caller, read by every later reset launch; NULL = each
 * instance's current size, the default). 0 = the winner keeps its maze and is only reset — the
 * variable-size envs' update_maze when `shape + 4 > max_shape` (simple_variable_maze_env.py:93-112,
 * toroidal_variable_maze_env.py:113-131), which leaves the maze as it is. A value the handle cannot
 * hold (even, < 5, > max_dim) counts as 0. */
int mz_set_regen_dims(mz_handle* h, const uint8_t* dims_dev);

/* rng of mz_generate_ex:
 *   MZ_RNG_PHILOX   Philox4x32 stream seed + env_id (as mz_generate): every random choice of the
 *                   reference is drawn uniformly over the same candidates (distribution parity).
 *   MZ_RNG_CPYTHON  CPython-exact: instance env_id gets the maze the reference builds with
 *                   `random.seed(seed + env_id); gen_maze((dim, dim), algo)` (toroidal:
 *                   gen_maze_no_border), bit for bit — MT19937 draws and CPython 3.10 set
 *                   iteration order emulated on the GPU (maze_generation.py:6-185). */
#define MZ_RNG_PHILOX 0
#define MZ_RNG_CPYTHON 1
int mz_generate_ex(mz_handle* h, const int32_t* env_ids_dev, int32_t n, const uint8_t* algo_dev,
                   int32_t algo_all, int32_t dim, uint64_t seed, int32_t rng, void* stream);

/* One CPython-exact maze for instance `env` from an explicit Python random state:
 * state_host[625] = random.getstate()[1] (624 MT19937 words + index), advanced in place exactly
 * as gen_maze((dim, dim), algo) would advance Python's global random (the caller writes it back
 * with random.setstate). Used by the single-env drop-in classes so that random.seed(s) before
 * construction gives the reference's maze (base_maze_env.py:78-97 draws six candidates from the
 * global stream). Synchronous. */
int mz_generate_state(mz_handle* h, int32_t env, int32_t dim, int32_t algo, uint32_t* state_host,
                      void* stream);

/* Reset every instance / a device list of instances (e.g. step's done_idx/done_count) and
 * write their reset observations into `out`. Replaces BaseMazeEnv.reset (base_maze_env.py:136-161).
 * A non-NULL count_dev is consumed: the kernel sets it to 0 once every workgroup has read it,
 * so the next mz_step_act may pass MZ_STEP_COUNT_ZEROED.
 * With regen_won != 0, listed instances whose last step terminated get a freshly generated maze
 * first (the trainer's win -> update_maze protocol, off_policy_trainer.py:190-202), using their
 * stored algorithm id and seed + env_id + (epoch << 32). */
int mz_reset_all(mz_handle* h, const mz_step_out* out, void* stream);
int mz_reset_list(mz_handle* h, const int32_t* idx_dev, const int32_t* count_dev,
                  int32_t max_count, int32_t regen_won, uint64_t seed, uint32_t epoch,
                  const mz_step_out* out, void* stream);

/* Auto-reset: reset every instance whose last step ended terminated|truncated (a per-instance
 * flag kept by the step; no device list needed) and write its reset observation into `out`.
 * With regen_won != 0 the instances that won get a new maze first (as mz_reset_list). */
int mz_reset_done(mz_handle* h, int32_t regen_won, uint64_t seed, uint32_t epoch,
                  const mz_step_out* out, void* stream);

/* One env step for all B instances. actions_dev: [B] int32 in 0..3 (BaseMazeEnv.ACTIONS);
 * a negative action means "observe only": no transition, outputs = observation of the current
 * state with reward 0 and terminated = truncated = 0 (used to step a subset of instances).
 * Replaces BaseMazeEnv.step (base_maze_env.py:163-210) with the move rule of
 * maze_view.move_agent (maze_view.py:167-197) and _get_obs/_find_best_next_cell (:116-122,
 * :224-262) / the Enrich window (maze_handler.py:4-99). */
int mz_step(mz_handle* h, const int32_t* actions_dev, const mz_step_out* out, void* stream);

/* flags of mz_step_ex / mz_step_act:
 *   MZ_STEP_COUNT_ZEROED  out->done_count is already 0 (skip the memset).
 *   MZ_STEP_AUTORESET     an instance whose previous step ended terminated|truncated is reset
 *                         by this launch instead of stepping (BaseMazeEnv.reset,
 *                         base_maze_env.py:136-161, same maze: the reference trainer's
 *                         env.reset() at the top of the next episode,
 *                         off_policy_trainer.py:153). Its action is ignored (actions_out = -1),
 *                         reward 0, terminated = truncated = 0, outputs = the reset
 *                         observation. One launch per vector step instead of step +
 *                         mz_reset_done. */
#define MZ_STEP_COUNT_ZEROED 1
#define MZ_STEP_AUTORESET 2
/* mz_step with flags. */
int mz_step_ex(mz_handle* h, const int32_t* actions_dev, const mz_step_out* out, int32_t flags,
               void* stream);

/* Fused act + step (one launch): each instance takes the epsilon-greedy action of mz_act
 * (below) and steps; actions_out_dev [B] (nullable) receives the actions taken. */
int mz_step_act(mz_handle* h, const float* eps_dev, float eps_all, const int64_t* greedy_dev,
                uint64_t seed, uint64_t counter, int32_t* actions_out_dev, const mz_step_out* out,
                int32_t flags, void* stream);

/* get_mask_direction(probs) for all instances: out4_dev [B][4] f32
 * (simple_maze_env.py:41-50, toroidal_maze_env.py:57-69). */
int mz_direction_mask(mz_handle* h, int32_t probs, float* out4_dev, void* stream);

/* Fused epsilon-greedy act (dqn_agent.py:104-116): for instance i, with u ~ U[0,1)
 * (Philox(seed, i, counter)), if u < eps[i] (eps_dev NULL = eps_all) sample from the
 * normalised get_mask_direction(probs=True) distribution, else take greedy_dev[i]
 * (NULL = always explore). Writes actions_dev [B] int32. */
int mz_act(mz_handle* h, const float* eps_dev, float eps_all, const int64_t* greedy_dev,
           uint64_t seed, uint64_t counter, int32_t* actions_dev, void* stream);

/* Expand n packed windows (window_bits layout) to f32 [n][3][15][15]. */
int mz_expand_window(const uint32_t* bits_dev, float* out_dev, int32_t n, void* stream);

/* Maze bank: regeneration on win (update_maze, simple_maze_env.py:81-94, called from
 * off_policy_trainer.py:190-202) copies a maze generated ahead of time instead of building one
 * inside mz_reset_done (one build is a ~1 ms serial chain: carve loop + two level-synchronous
 * BFS; a copy is a few microseconds). Two banks of `slots` mazes per algorithm in algo_mask
 * (bit a = algorithm id a), all of size `dim`; the caller consumes one (mz_bank_use) while it
 * refills the other (mz_bank_fill, e.g. on a side stream ordered after the consuming launches).
 * Mazes: Philox seed ^ ((3*bank + algo + 1) << 56) + slot + (fill epoch << 32). An exhausted
 * bank, or an instance whose algorithm / size the bank lacks, falls back to building in place. */
int mz_bank_create(mz_handle* h, int32_t slots, int32_t dim, uint32_t algo_mask);
/* The same for a list of ndims (<= MZ_BANK_MAX_DIMS) distinct maze sizes: `slots` mazes per
 * (algorithm, size) — the variable-size envs (config 5: toroidal 17..79, instance i of size
 * dims[i mod n]); a win copies a maze of the instance's own size. Size index di keys its slots'
 * Philox seeds with di << 48 (di = 0: mz_bank_create's). */
int mz_bank_create_dims(mz_handle* h, int32_t slots, const int32_t* dims, int32_t ndims,
                        uint32_t algo_mask);
/* mz_bank_create_dims whose slots are best-of-`candidates` mazes (1..MZ_MAX_CANDIDATES): every
 * refilled slot is the easiest of `candidates` mazes by McClendon difficulty, the first on ties —
 * the reference's generate_maze selection for the new maze of a win (base_maze_env.py:78-97,
 * toroidal_maze_env.py:40-54, via update_maze at off_policy_trainer.py:202 / ppo_trainer.py:96).
 * Candidate c of slot j of a fill: Philox key + j * candidates + c + (epoch << 32) with the
 * block's key as mz_bank_fill's (candidates = 1: mz_bank_create_dims exactly). Needs the
 * difficulty kernel's LDS plan (max_dim <= 91 euclidean, <= 89 toroidal) when candidates > 1;
 * the K * candidates candidate mazes live in scratch owned by the handle. */
int mz_bank_create_ex(mz_handle* h, int32_t slots, const int32_t* dims, int32_t ndims,
                      uint32_t algo_mask, int32_t candidates);
/* Rebuild the slots of `bank` consumed since its last fill (every slot on the first fill). */
int mz_bank_fill(mz_handle* h, int32_t bank, uint64_t seed, void* stream);
/* Inspect one bank slot (synchronous; tests): the grid (0 wall, 1 floor, 2 goal) into
 * grid_host [N][N] (N = the slot's size, <= max_dim) and (start r, start c, goal r, goal c). */
int mz_bank_slot_grid(mz_handle* h, int32_t bank, int32_t algo, int32_t size_index, int32_t slot,
                      uint8_t* grid_host, int32_t* info4_host);
/* Bank consumed by later mz_reset_done(regen_won) launches; -1 = none (build in place). */
int mz_bank_use(mz_handle* h, int32_t bank);
/* Consumed-slot counters of `bank` per algorithm id and size index -> out3_dev [3][ndims] int32
 * (device; [3] for a single-size bank). */
int mz_bank_consumed(mz_handle* h, int32_t bank, int32_t* out3_dev, void* stream);

/* Checkpoint / resume of a handle's env state (the reference has none; its envs keep
 * their mazes in Python lists, simple_maze_env.py:34,91). One device buffer holds a 256-B header
 * (magic "MZST", version, B, P, toroidal, enrich, the bank geometry, the active bank and its fill
 * epochs) and every per-instance array of the handle — cell words (maze, BFS table, visit counts
 * and tags), open / visited plane strips, meta, position / step / current-cell words, algorithm
 * ids, last-terminated flags — plus, when the handle has a maze bank, both banks with their
 * consumed-slot counters. mz_state_bytes: the buffer size; mz_state_save: device-to-device copies
 * on `stream`; mz_state_load: validates the header against the handle (same num_envs, max_dim,
 * toroidal, enrich; the same bank geometry, created with mz_bank_create*; MZ_EINVAL otherwise),
 * then copies back and re-activates the saved bank. Stepping a loaded handle continues
 * bit-exactly where the saved one stood. */
#define MZ_STATE_HEADER_BYTES 256
int mz_state_bytes(mz_handle* h, uint64_t* bytes_out);
int mz_state_save(mz_handle* h, void* dst_dev, uint64_t bytes, void* stream);
int mz_state_load(mz_handle* h, const void* src_dev, uint64_t bytes, void* stream);

/* Fused conv stem of the DQN/DDQN Q-network for acting (dqn_agent.py:19-57 forward,
 * ddqn_agent.py:18-52): from n packed windows (window_bits layout) and obs6 [n][6] f32, writes
 * feat_dev [n][ld] bf16 = [MaxPool2(Dropout(LeakyReLU(Conv3x3(window) + b))) (1,568 values,
 * position-major: element q*32 + c = channel c at pooled position q; torch's flatten order is
 * c*49 + q, so fc1's weight columns are permuted once by the caller) | obs6 (6) | zeros], the
 * input row of the first Linear layer.
 * conv_w_dev f32 [32][3][3][3], conv_b_dev f32 [32]; drop_p = 0 (DQN) or the Dropout p (DDQN in
 * train mode), masks drawn from (seed, counter); ld in 1576..1600, multiple of 8. */
int mz_q_front(const uint32_t* bits_dev, const float* obs6_dev, int32_t n, const float* conv_w_dev,
               const float* conv_b_dev, float drop_p, uint64_t seed, uint64_t counter,
               uint16_t* feat_dev, int32_t ld, void* stream);

/* mz_q_front over a row list: output row i is instance rows_dev[i] (i < n) of bits_dev / obs6_dev;
 * with count_dev (nullable) the rows i < min(n, *count_dev), the length read on the device (the
 * stem can run before the caller knows the list's length). With the list of mz_greedy_rows the
 * acting forward runs over the rows that act greedily only (dqn_agent.py:104-116 evaluates
 * source_net(state) only when `sample >= eps`). */
int mz_q_front_rows(const uint32_t* bits_dev, const float* obs6_dev, const int32_t* rows_dev,
                    const int32_t* count_dev, int32_t n, const float* conv_w_dev,
                    const float* conv_b_dev, float drop_p, uint64_t seed, uint64_t counter,
                    uint16_t* feat_dev, int32_t ld, void* stream);

/* Greedy-row list of the next fused act (mz_act / mz_step_act with the same eps, seed, counter;
 * dqn_agent.py:104-116 draws `sample = random.random()` first and acts greedily iff
 * sample >= eps): rows_dev[0 .. count) = the instances i < n that will take greedy_dev[i], in
 * increasing order; count_dev [1] int32 (device) and, if count_host is not NULL, the same count
 * into mapped host memory (mz_host_alloc) for the caller's GEMM sizes. scratch_dev: int32
 * [ceil(n / 1024)]. Two launches, no atomics: the list is deterministic. */
int mz_greedy_rows(const float* eps_dev, float eps_all, uint64_t seed, uint64_t counter, int32_t n,
                   int32_t* scratch_dev, int32_t* rows_dev, int32_t* count_dev,
                   int32_t* count_host, void* stream);

/* The same conv stem in f32 for the LEARNER update (optimize_model, dqn_agent.py:121-157,
 * ddqn_agent.py:113-152; forward dqn_agent.py:47-57), forward and backward, from packed windows:
 * feat_dev [n][ld] f32 = [MaxPool2(Dropout(LeakyReLU(Conv3x3(window) + b))) in torch's flatten
 * order (c*49 + q) | obs6], ld >= 1574, i.e. the f32 input of fc.0. drop_p = 0 (DQN) or the
 * Dropout p (DDQN); the mask key is read from rng_dev (a device u64 the caller advances between
 * calls, so a captured HIP graph draws fresh masks on every replay) mixed with `salt`.
 * code_dev [n][1568] u8 (NULL when no backward follows): per feature the pooled argmax (bits
 * 0-1) and its gradient class (bits 2-3: 0 dropped, 1 kept with a > 0, 2 kept with a <= 0). */
int mz_stem_forward(const uint32_t* bits_dev, const float* obs6_dev, int32_t n,
                    const float* conv_w_dev, const float* conv_b_dev, float drop_p,
                    const uint64_t* rng_dev, uint32_t salt, float* feat_dev, int32_t ld,
                    uint8_t* code_dev, void* stream);
/* Conv weight / bias gradients from the gradient of the stem output gfeat_dev [n][ld] f32 (its
 * first 1,568 columns) and the forward's code bytes: dw_dev [32][3][3][3], db_dev [32] f32
 * (overwritten). partial_dev: workspace of mz_stem_workspace_floats(n) floats. */
int mz_stem_backward(const uint32_t* bits_dev, const uint8_t* code_dev, const float* gfeat_dev,
                     int32_t ld, int32_t n, float drop_p, float* partial_dev, float* dw_dev,
                     float* db_dev, void* stream);
/* mz_stem_backward that also advances the device u64 rng_advance_dev by one after the gradient
 * launches (NULL: nothing advanced): a learner whose nets read one dropout counter in every
 * forward of an update moves it on from the backward, with no launch of its own per forward. */
int mz_stem_backward_ex(const uint32_t* bits_dev, const uint8_t* code_dev, const float* gfeat_dev,
                        int32_t ld, int32_t n, float drop_p, float* partial_dev, float* dw_dev,
                        float* db_dev, uint64_t* rng_advance_dev, void* stream);
int mz_stem_workspace_floats(int32_t n);

/* The learner's parameter update: grad.clamp_(-clamp, clamp) on every parameter, then one
 * torch.optim.AdamW step (dqn_agent.py:152-157, ddqn_agent.py:148-152: AdamW(lr) with the
 * defaults betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2 — the eager single-tensor formula)
 * over a flat f32 parameter buffer param_dev with its moment buffers exp_avg_dev /
 * exp_avg_sq_dev (same length, 16-byte aligned). Gradients come as nseg (<= 16) device segments:
 * grads_dev[k] (host array of device pointers, each 16-byte aligned) holds the gradient of flat
 * elements [sum(seg_len[:k]), sum(seg_len[:k+1])), seg_len[k] a multiple of 4; each is scaled by
 * grad_scale before the clamp (1/N after an all-reduce sum) and, if write_grad, written back
 * clamped. lr_dev: f32 learning rate on the device (the cosine schedule writes it); step_dev:
 * f32 step counter on the device, incremented by this call before the bias corrections (so a
 * captured HIP graph advances it on every replay). One launch over every parameter. */
/* nn.LeakyReLU(slope) in place on n bf16 values (the acting head's hidden layers, dqn_agent.py
 * :52-57): x > 0 ? x : x * slope in f32, rounded to nearest even — torch's leaky_relu_ on bf16
 * element for element. n a multiple of 8, x_dev 16-byte aligned. */
int mz_leaky_relu_bf16(uint16_t* x_dev, int64_t n, float slope, void* stream);

/* Column sums out_dev[c] = sum_{r < n} g_dev[r * ld + c], c < m, f32: the Linear bias gradient
 * db = dY^T 1 of the learner updates (the bias term of optimize_model's backward,
 * dqn_agent.py:150 / ppo_agent.py:235). m and ld multiples of 4, buffers 16-byte aligned;
 * fixed summation order (deterministic). */
int mz_colsum_f32(const float* g_dev, int32_t n, int32_t m, int32_t ld, float* out_dev,
                  void* stream);

/* One learner update's replay sample (ReplayMemory.sample, replay_memory.py:17-18, drawn as
 * indices on the device): rows idx_dev[i] (i < b, int64, clamped into [0, capacity)) of the state
 * arrays obs6 f32 [capacity][6] / window bits int32 [capacity][22] and of the next-state arrays
 * go to rows i and b + i of out_s6_dev f32 [2b][6] / out_sw_dev int32 [2b][22] (state rows, then
 * next-state rows), actions int64 and rewards f32 to out_a_dev / out_r_dev [b]. */
int mz_replay_gather(const int64_t* idx_dev, int32_t b, int64_t capacity,
                     const float* s6_dev, const int32_t* sw_dev, const int64_t* a_dev,
                     const float* r_dev, const float* s6n_dev, const int32_t* swn_dev,
                     float* out_s6_dev,
                     int32_t* out_sw_dev, int64_t* out_a_dev, float* out_r_dev, void* stream);

/* The PPO clipped surrogate with the reference's [b, b] broadcast (ppo_agent.py:188-197, clip
 * 0.3 there): for every column i, part_dev[i] = sum_j min(r a_i, clamp(r, 1-clip, 1+clip) a_i)
 * and dsum_dev[i] = sum_j r * w with r = exp(lp_new[i] - lp_old[j]) and w torch's gradient
 * routing through min / clamp (1/2 + 1/2 [inside] on ties, 1 where r a_i is the smaller, [inside]
 * otherwise). The loss is sum(part) / b^2 and dL/dlp_new[i] = a_i dsum[i] / b^2. All f32 [b]. */
int mz_pair_surrogate(const float* lp_new_dev, const float* lp_old_dev, const float* adv_dev,
                      int32_t b, float clip, float* part_dev, float* dsum_dev, void* stream);

/* The DQN/DDQN optimizer step (dqn_agent.py:152-157, ddqn_agent.py:148-152: grad.clamp_(-c, c)
 * per parameter, then torch.optim.AdamW) as one launch over a flat f32 parameter buffer whose
 * segment k (length seg_len[k], a multiple of 4) has its gradient at grads_dev[k] (host array of
 * nseg <= 16 device pointers). lr_dev: device f32 learning rate. step_dev: device f32 [1], the
 * step count, advanced by one by the call itself on `stream` (a one-thread launch behind the
 * update: a captured graph advances it per replay). write_grad: store the clamped,
 * grad_scale-scaled gradient back (clamp_ in place). */
int mz_adamw_flat(float* param_dev, float* exp_avg_dev, float* exp_avg_sq_dev,
                  const float* const* grads_dev, const int64_t* seg_len, int32_t nseg,
                  const float* lr_dev, float* step_dev, double beta1, double beta2, double eps,
                  double weight_decay, float clamp, float grad_scale, int32_t write_grad,
                  void* stream);

/* Set the per-instance algorithm ids used by regeneration (BaseMazeEnv.ALGORITHM is global in
 * the reference, base_maze_env.py:17,60-64; here it is per instance). algo_dev [B] or NULL. */
int mz_set_algorithm(mz_handle* h, const uint8_t* algo_dev, int32_t algo_all, void* stream);

/* Per-instance maze metadata into meta_dev [B][6] int32: N, start r, start c, goal r, goal c,
 * max_steps (the attributes maze_shape/_start_pos/_target_location/max_steps_taken). */
int mz_get_meta(mz_handle* h, int32_t* meta_dev, void* stream);

/* PPO discounted returns (ppo_agent.py:170-179) for n episodes on the device: episode k is row
 * rows_dev[k] of rew_dev (float64, leading dim ld) with length lens_dev[k]; out_dev[k*ldo + t] =
 * float32(sum_j gamma^j r[t+j]) accumulated backwards in float64 like the reference's loop. */
int mz_discounted_returns(const double* rew_dev, int32_t ld, const int32_t* rows_dev,
                          const int32_t* lens_dev, int32_t n, double gamma, float* out_dev,
                          int32_t ldo, void* stream);

/* McClendon difficulty of a maze (host computation, synchronous): ComplexityEvaluation(maze,
 * start, goal).difficulty_of_maze() (maze_complexity_evaluation.py:38-329) for a euclidean grid
 * (toroidal mazes: pass the bordered (N+2) grid, as gen_maze_no_border does, :37-56).
 * Used by get_maze_difficulty (base_maze_env.py:99-105) and best-of-6 generation (:78-97). */
int mz_difficulty(const uint8_t* grid_host, int32_t h, int32_t w, int32_t sr, int32_t sc,
                  int32_t gr, int32_t gc, double* out_host);

/* McClendon difficulty and complexity together (complexity_of_maze :311-317 = log of the sum of
 * the branch complexities; difficulty as mz_difficulty). Either output may be NULL. Host,
 * synchronous. */
int mz_maze_complexity(const uint8_t* grid_host, int32_t h, int32_t w, int32_t sr, int32_t sc,
                       int32_t gr, int32_t gc, double* difficulty_out, double* complexity_out);

/* McClendon difficulty of resident mazes on the GPU, one workgroup per maze (replaces the
 * per-maze host ComplexityEvaluation(...).difficulty_of_maze() calls of best-of-6 generation,
 * base_maze_env.py:84-95, maze_complexity_evaluation.py:38-329). For the listed instances
 * (env_ids_dev NULL = all B): out_dev [n][2] float64 = {prod, sum}, the reference's product
 * prod_b (C_b + 1) * C_0 and sum sum_b C_b + C_0 BEFORE math.log (the caller takes the log with
 * the C library, as the reference: difficulty = log(prod), complexity = log(sum)), each hallway
 * summed in the order networkx's subgraph view iterates its CPython set (bit-exact with the
 * reference); a toroidal handle's maze is scored as its bordered (N + 2)^2 maze with start / goal
 * shifted by +1, as the reference scores it (off_policy_trainer.py:194-196). status_dev [n]
 * int32: 0 ok, 1 not a perfect maze (cycles / unreachable squares), 2 outside the kernel's cases
 * (open border squares, straight goal square, all solution points junctions, more points than
 * the LDS plan holds, a hallway of more than 63 view nodes), 3 invalid (start == goal, bad id,
 * log domain) — the caller computes every nonzero-status maze with mz_difficulty (toroidal: on
 * the bordered grid). Asynchronous on `stream`. Returns MZ_EINVAL_SHAPE when the evaluated grid's
 * pitch exceeds the kernel's LDS plan (odd pitches: P > 91; toroidal P > 89 — the bordered grid
 * is P + 2; tests/test_abi.py derives both limits from the plan). */
int mz_difficulty_batch(mz_handle* h, const int32_t* env_ids_dev, int32_t n, double* out_dev,
                        int32_t* status_dev, void* stream);
/* The order-free McClendon screen (csrc/mz_screen.hip; the best-of-C selection's first stage) of
 * the listed euclidean instances (NULL = all B): out_dev [n][2] float64 = {prod, e} — the product
 * prod_b (C_b + 1) * C_0 of maze_complexity_evaluation.py:319-329 summed in an order of its own,
 * and a rigorous bound e on |prod_ref - prod| / prod for the reference's evaluation order (which
 * mz_difficulty_batch reproduces); status_dev [n] int32: 0 ok, 2 declined (not a perfect maze on
 * the odd lattice with a dead-end goal, or beyond the LDS plan). One wave per maze. */
int mz_screen_batch(mz_handle* h, const int32_t* env_ids_dev, int32_t n, double* out_dev,
                    int32_t* status_dev, void* stream);

/* The reference's maze-metric suite (MetricsCalculator, metrics_calculator.py:11-133, as used by
 * generation_algos_metrics_evaluations.py:33-45) for the listed euclidean instances (NULL = all B),
 * computed on the GPU from the instances' mazes: out_dev [n][6] float64 = L, DE, D, AC, FDE, BDE
 * of the solution path (calculate_L / calculate_DE / calculate_D / calculate_DE_sub). */
int mz_maze_metrics(mz_handle* h, const int32_t* env_ids_dev, int32_t n, double* out_dev,
                    void* stream);

/* Synchronous host snapshots for the single-env drop-in classes. */
int mz_query(mz_handle* h, int32_t env, mz_env_info* info_host);
int mz_get_grid(mz_handle* h, int32_t env, uint8_t* grid_host /* [n][n] */);

/* Page-locked host memory mapped into the device's address space (hipHostMalloc, mapped +
 * coherent): kernels read and write it through *dev_out. The single-env drop-ins keep their
 * action and per-step outputs there, so one reference step() (base_maze_env.py:163-210) is one
 * launch + one stream synchronisation, with no device<->host copies. Free with mz_host_free. */
int mz_host_alloc(uint64_t bytes, int32_t device, void** host_out, void** dev_out);
int mz_host_free(void* host);

/* ---- Vectorised trainer bookkeeping (mazerl/trainers/vector_trainer.py; the training loop of
 * NeuralOffPolicyTrainer.train, lib/trainers/off_policy_trainer.py:144-225, over n instances).
 * The loop waits once per vector step for the greedy-row count; these calls keep the launches
 * behind that wait few. */

/* After a vector step: steps_done += 1, = 0 where terminated (off_policy_trainer.py:192, per
 * instance); eps_out = eps_final + (eps_start - eps_final) * exp(-steps_done / eps_decay) in f32
 * (dqn_agent.py:118-119 calculate_epsilon, as the learner's torch expression rounds it);
 * wins += #terminated, episodes += #(terminated | truncated) (int64 device counters, nullable);
 * and the greedy-row list of the NEXT fused act (seed, counter, eps_out): rows_dev / count_dev as
 * mz_greedy_rows. scratch_dev: int32 [ceil(n / 1024)]. */
int mz_trainer_tick(const uint8_t* term_dev, const uint8_t* trunc_dev, float* steps_done_dev,
                    double eps_start, double eps_final, double eps_decay, float* eps_out_dev,
                    int64_t* wins_dev, int64_t* episodes_dev, uint64_t seed, uint64_t counter,
                    int32_t n, int32_t* scratch_dev, int32_t* rows_dev, int32_t* count_dev,
                    void* stream);

/* greedy_dev[rows_dev[i]] = argmax_a q_dev[i][a] (first maximum, torch.argmax) for
 * i < min(*count_dev, m): the acting forward's bf16 Q rows [m][ldq] (dqn_agent.py:113-116
 * `.max(1)[1]`) scattered to the listed instances; the list length is read on the device. */
int mz_greedy_scatter(const uint16_t* q_dev, int32_t ldq, const int32_t* rows_dev,
                      const int32_t* count_dev, int32_t m, int64_t* greedy_dev, void* stream);

/* bf16 copy of the acting head's three Linear layers (dqn_agent.py:47-57 / ddqn_agent.py:40-52
 * fc): w_l f32 [out_l][in_l] -> dw_l bf16 (round to nearest even, torch's .to(bfloat16)); fc1's
 * first conv_out columns permuted from torch's channel-major flatten (c * Q + q, Q = conv_out /
 * conv_ch) to the fused stem's position-major order (q * conv_ch + c), rows padded with zeros to
 * ld0 (in0 <= 2048); biases b_l -> db_l. One launch. */
int mz_head_bf16(const float* w0, const float* b0, const float* w1, const float* b1,
                 const float* w2, const float* b2, int32_t out0, int32_t in0, int32_t out1,
                 int32_t in1, int32_t out2, int32_t in2, int32_t ld0, int32_t conv_out,
                 int32_t conv_ch, uint16_t* dw0, uint16_t* db0, uint16_t* dw1, uint16_t* db1,
                 uint16_t* dw2, uint16_t* db2, void* stream);

/* Replay ring push (lib/replay_memory.py:14 push, a vector step at once): ring rows ptr ..
 * ptr + n - 1 (mod capacity) of s6 f32 [C][obs_dim], sw int32 [C][window_words], a int64 [C]
 * (from int32 actions), r f32 [C], s6n, swn <- the n source rows; a NULL source leaves its array
 * untouched (the state half can be written before the env step overwrites the observation). */
int mz_replay_push(int32_t n, int64_t capacity, int64_t ptr, const float* obs6_src,
                   const int32_t* bits_src, const int32_t* act_src, const float* rew_src,
                   const float* obs6n_src, const int32_t* bitsn_src, float* s6_dev,
                   int32_t* sw_dev, int64_t* a_dev, float* r_dev, float* s6n_dev,
                   int32_t* swn_dev, int32_t obs_dim, int32_t window_words, void* stream);

/* n uniform replay rows (random.sample of replay_memory.py:17, with replacement) among the newest
 * n_avail ring rows ending at row `newest`: out_dev[i] = (newest - floor(u_i * n_avail)) mod
 * capacity, u_i a 53-bit uniform from Philox(seed, i, counter). */
int mz_replay_sample_idx(uint64_t seed, uint64_t counter, int64_t newest, int64_t n_avail,
                         int64_t capacity, int64_t* out_dev, int32_t n, void* stream);

/* Q-learning loss of optimize_model (dqn_agent.py:129-147, ddqn_agent.py:121-143) from the nets'
 * f32 output rows: for i < b, Q(s,a) = q_dev[i][action_dev[i]]; V(s') = q_tgt_dev[i][argmax_a
 * q_next_dev[i][a]] (DDQN; first maximum) or max_a q_tgt_dev[i][a] (DQN: q_next_dev NULL);
 * diff_dev[i] = Q(s,a) - (V(s') * gamma + reward_dev[i]) — no terminal masking (the reference
 * bootstraps terminal transitions); *loss_dev = mse_loss (mean) = sum diff^2 / b.
 * Row strides ldq / ldn / ldt in floats (>= 4). One workgroup. */
int mz_q_loss(const float* q_dev, int32_t ldq, const float* q_next_dev, int32_t ldn,
              const float* q_tgt_dev, int32_t ldt, const int64_t* action_dev,
              const float* reward_dev, double gamma, int32_t b, float* loss_dev, float* diff_dev,
              void* stream);

/* Its gradient w.r.t. q rows [rows][4] (contiguous; rows >= b — DDQN's stacked s' rows — get 0):
 * dq[i][action[i]] = diff[i] * (2 / b) * (*grad_dev), 0 elsewhere. */
int mz_q_loss_backward(const float* grad_dev, const float* diff_dev, const int64_t* action_dev,
                       int32_t b, int32_t rows, float* dq_dev, void* stream);

/* The Q head and the loss of optimize_model in one launch, from the second hidden layer's
 * pre-activation rows z2 (f32, row stride lds / ldt floats, `hidden` columns, a multiple of 4) of
 * the source and the target net: h = act(z2) (act 0: LeakyReLU(0.01), DQN; 1: ReLU, DDQN),
 * q = W3 h + b3 (fc3: W3 [4][hidden], b3 [4]); with `stacked` the source rows are DDQN's [s; s']
 * (2b rows: V(s') = q_t[argmax q_s(s')], first maximum), else b rows and V(s') = max q_t; then
 * diff_dev / *loss_dev exactly as mz_q_loss (dqn_agent.py:129-147, ddqn_agent.py:121-143).
 * part_dev: mz_head_loss_workspace_floats(b) floats (one per concurrently running call);
 * ticket_dev: unused since round 5 (the per-workgroup partials are summed by a second launch on
 * `stream`), may be NULL. Replaces the activation, fc3 and loss launches of both nets. */
int mz_head_loss_workspace_floats(int32_t b);
int mz_head_loss(const float* z2s_dev, int32_t lds, const float* w3s_dev, const float* b3s_dev,
                 const float* z2t_dev, int32_t ldt, const float* w3t_dev, const float* b3t_dev,
                 int32_t hidden, int32_t act, int32_t stacked, const int64_t* action_dev,
                 const float* reward_dev, double gamma, int32_t b, float* part_dev,
                 uint32_t* ticket_dev, float* loss_dev, float* diff_dev, void* stream);

/* Its backward through fc3 and the activation for the source rows i < b: dz2_dev[i][j] =
 * act'(z2[i][j]) * g_i W3[a_i][j], g_i = diff[i] * (2 / b) * (*grad_dev) (rows >= b untouched),
 * and per block of rows the partial sums of dW3 (row-major [4][hidden]) and db3 [4] into part_dev
 * ([blocks][4 hidden + 4], mz_head_loss_backward_workspace_floats floats): their column sums
 * (mz_colsum_f32 over blocks rows of 4 hidden + 4) are fc3's weight and bias gradients. */
int mz_head_loss_backward_workspace_floats(int32_t b, int32_t hidden);
int mz_head_loss_backward(const float* grad_dev, const float* diff_dev, const int64_t* action_dev,
                          int32_t b, const float* z2s_dev, int32_t lds, const float* w3s_dev,
                          int32_t hidden, int32_t act, float* dz2_dev, int32_t ldd,
                          float* part_dev, void* stream);

/* PPO's optimizer step (ppo_agent.py:232-236, optimize_model): clip_grad_norm_(params, max_norm)
 * (coef = min(max_norm / (||g||_2 + 1e-6), 1) over every gradient, the gradients scaled in place;
 * max_norm <= 0: no clipping), then AdamW (torch's defaults: betas, eps, weight_decay given) with
 * a learning rate per parameter group — segment k of the flat buffer (mz_adamw_flat's layout)
 * uses lr_dev[seg_group[k]] (ppo_agent.py's three groups: actor lr, critic lr, their mean for
 * the conv stem). step_dev is incremented on the device (capturable). scratch_dev: >= 513
 * floats. Three launches. */
int mz_adamw_groups(float* param_dev, float* exp_avg_dev, float* exp_avg_sq_dev,
                    const float* const* grads_dev, const int64_t* seg_len,
                    const int32_t* seg_group, int32_t nseg, const float* lr_dev, float* step_dev,
                    double beta1, double beta2, double eps, double weight_decay, float max_norm,
                    float* scratch_dev, void* stream);

/* ---- Config 5's PPO rollout on the device (VectorPPOTrainer; no host round trip per step) ----
 * B instances, per-instance episode records [B][L] at the instance's own step index t_dev[i]
 * (L > the longest possible episode). Replaces, per instance, PPOAgent.do_episode's loop
 * (agents/ppo_agent.py:143-169) and PPOTrainer.train's Buffer.add (lib/trainers/ppo_trainer.py
 * :15-46, :66-67). */

/* ActorCriticNet.act (ppo_agent.py:55-68) from the f32 actor logits [B][ldl] and critic values
 * [B] (stride ldv): softmax as torch forms it for a 4-wide row, one draw per instance (inverse
 * CDF of a Philox uniform: P(a) = softmax(logits)[a], torch.multinomial's distribution), the
 * draw's log-prob log(p[a]); records obs6, the 22 window-bit words, action (int64), log-prob and
 * value at [i][t_dev[i]] (do_episode's appends, :150-156) and writes the action to act_out_dev
 * (int32, mz_step's input). */
int mz_ppo_act(const float* logits_dev, int32_t ldl, const float* value_dev, int32_t ldv,
               const float* obs6_dev, const uint32_t* bits_dev, int32_t B, int32_t L, uint64_t seed,
               uint64_t counter, const int32_t* t_dev, float* rec_s6_dev, uint32_t* rec_w_dev,
               int64_t* rec_a_dev, float* rec_lp_dev, float* rec_v_dev, int32_t* act_out_dev,
               void* stream);

/* After mz_step: the float64 reward at [i][t_dev[i]] (rewards.append, :158), t_dev[i] += 1, and
 * for every instance whose step ended (terminated | truncated, :161): t_dev[i] = 0, stats_dev
 * [0] += 1 (episodes), [1] += terminated (wins), and — for episodes of >= 2 steps (a 1-step
 * episode's returns are NaN: torch.std of one element; counted in stats_dev[2] instead) — an
 * entry in the finished list (instance fin_id, pool row fin_off, length fin_len; instance order)
 * placed after the pool's current *pool_fill_dev rows; *pool_fill_dev and the monotonic
 * *pool_total_dev grow by the listed rows. stats_dev[3] counts unfinished episodes that reached
 * L steps (their records would leave the [B][L] buffers; t_dev stays at L - 1): the caller sizes
 * L past every max_steps + 1 and treats a nonzero count as an error. stats_dev is int64[4].
 * One workgroup. */
int mz_ppo_scan(const double* reward64_dev, const uint8_t* term_dev, const uint8_t* trunc_dev,
                int32_t B, int32_t L, int32_t* t_dev, double* rec_r_dev, int32_t* fin_id_dev,
                int64_t* fin_off_dev, int32_t* fin_len_dev, int32_t* fin_count_dev,
                int64_t* pool_fill_dev, int64_t* pool_total_dev, int64_t* stats_dev,
                void* stream);

/* For every listed episode: calculate_returns (ppo_agent.py:171-181: acc = r + acc * gamma
 * backwards in float64, float32, (R - mean) / std, unbiased std) and calculate_advantages
 * (:183-186: A = R - V, (A - mean) / (std + 1e-8)) — sums in float64, mean / std rounded to
 * float32 — and the episode's rows (obs6, window bits, action, log-prob, advantage, return)
 * into the pool columns at its rows (rows past `capacity` are not written: the caller checks
 * *pool_fill_dev <= capacity). One workgroup per episode. */
int mz_ppo_finish(const double* rec_r_dev, const float* rec_s6_dev, const uint32_t* rec_w_dev,
                  const int64_t* rec_a_dev, const float* rec_lp_dev, const float* rec_v_dev,
                  int32_t B, int32_t L, const int32_t* fin_id_dev, const int64_t* fin_off_dev,
                  const int32_t* fin_len_dev, const int32_t* fin_count_dev, double gamma,
                  int64_t capacity, float* pool_s6_dev, uint32_t* pool_w_dev, int64_t* pool_a_dev,
                  float* pool_lp_dev, float* pool_adv_dev, float* pool_ret_dev, void* stream);

/* The PPO minibatch loss in three launches (ppo_agent.py:188-203 through ActorCriticNet.evaluate,
 * :55-66, and optimize_model's total = policy + 0.5 value, :222-224): for b rows of 4 action
 * logits (row stride ldl), value (stride ldv), action, old log-prob, advantage, return and the
 * entropy coefficient (device scalar): softmax, the action's log_softmax, entropy
 * -sum p log(p + 1e-8), the clipped surrogate over the reference's [b, b] ratio broadcast
 * (mz_pair_surrogate), total = -(surrogate + coef * mean entropy) + 0.5 * mean((v - ret)^2) into
 * loss_dev[0], and d total / d logits (dlogits_dev, row stride ldg) and d total / d value
 * (dvalue_dev, stride ldvg). scratch_dev: 12 b floats. Sums in a fixed order (deterministic). */
int mz_ppo_head_loss(const float* logits_dev, int32_t ldl, const float* value_dev, int32_t ldv,
                     const int64_t* action_dev, const float* lp_old_dev, const float* adv_dev,
                     const float* ret_dev, const float* coef_dev, int32_t b, float clip,
                     float* scratch_dev, float* loss_dev, float* dlogits_dev, int32_t ldg,
                     float* dvalue_dev, int32_t ldvg, void* stream);

/* ---- The DQN / DDQN acting forward, f32-accurate on the bf16 MFMA (mz_qact.hip) -------------
 * Replaces, per acting row, source_net(state).max(1)[1] (dqn_agent.py:113-116; the nets of
 * dqn_agent.py:19-57 / ddqn_agent.py:18-52 at the reference's sizes: Conv2d(3, 32, 3, p 1),
 * 1,574 -> 1,024 -> 512 -> 4). Every GEMM operand is split into bf16 hi + lo and each product
 * summed as hi*hi + hi*lo + lo*hi in f32 (~2^-16 relative): the f32 argmax at bf16-MFMA speed. */

/* fc1's weight [1024][1574] (torch layout) and fc2's [512][1024] f32 -> the hi / lo bf16 images
 * mz_qact reads, in MFMA fragment order (a wave's operand for one K chunk contiguous): w1 1024 x 1600
 * elements (features in the kernel's order, zero pad), w2 512 x 1024. Every pointer 16-B aligned (MZ_EINVAL otherwise). */
int mz_qact_prepare(const float* fc1_w_dev, const float* fc2_w_dev, uint16_t* w1_hi_dev,
                    uint16_t* w1_lo_dev, uint16_t* w2_hi_dev, uint16_t* w2_lo_dev, void* stream);

/* Q values and greedy actions of min(n, *count_dev) rows (count_dev NULL: n): row i is instance
 * rows_dev[i] (rows_dev NULL: instance i) of bits_dev [B][22] / obs6_dev [B][6]. Conv weight
 * [32][3][3][3] / bias, fc1 bias [1024], fc2 bias [512], fc3 weight [4][512] / bias [4] f32;
 * relu: 1 for DDQN's second activation (ReLU), 0 for DQN's LeakyReLU; drop_p > 0: DDQN's
 * train-mode Dropout after the conv activation (counter hash of seed / counter, row, feature).
 * h1_dev: workspace of mz_qact_workspace_floats(n) f32 (fc1's output rows [n][1024], then the
 * conv stem's bf16 hi / lo feature tiles: the stem runs once per 64 rows, k_qconv, and fc1 reads
 * them, k_qfc1). Outputs: greedy_dev[instance] = first argmax (int64; NaN as torch.argmax),
 * q_out_dev [n][4] f32 (either may be NULL). No host synchronisation. */
int64_t mz_qact_workspace_floats(int32_t n);
int mz_qact(const uint32_t* bits_dev, const float* obs6_dev, const int32_t* rows_dev,
            const int32_t* count_dev, int32_t n, const float* conv_w_dev, const float* conv_b_dev,
            const uint16_t* w1_hi_dev, const uint16_t* w1_lo_dev, const float* b1_dev,
            const uint16_t* w2_hi_dev, const uint16_t* w2_lo_dev, const float* b2_dev,
            const float* w3_dev, const float* b3_dev, int32_t relu, float drop_p, uint64_t seed,
            uint64_t counter, float* h1_dev, int64_t* greedy_dev, float* q_out_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif
