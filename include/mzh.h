/*
 * mzh.h -- C ABI of libmzh.so: MI355X-native (gfx950 HIP) batched MuZero-MCTS + Tower-of-Hanoi.
 *
 * The reference (A-Andrews/Muzero-Hanoi) is pure Python; its "plugin boundary" is the duck-typed
 * Python API that training_main.py / Muzero.py / the acting scripts call.  Each entry point below
 * replaces one of those interfaces (cited file:line); the Python host layer in muzero-hanoi_amd/
 * binds them with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every buffer argument is a DEVICE pointer owned by the caller (e.g. a torch tensor's
 *    data_ptr()), except where "host" is written.  Shapes are row-major; B = batch of roots/envs.
 *  - Calls are asynchronous and stream-ordered on `stream` (a hipStream_t; NULL = null stream).
 *  - Every function returns an int status (MZH_OK = 0, negative on error) and never throws;
 *    mzh_last_error() returns a thread-local message for the last failure.
 *  - An engine is bound to one device and is not re-entrant across threads (one engine per
 *    device/stream, like the reference's single MCTS instance, MCTS/mcts.py:23).
 *  - No CPU fallback exists: without a HIP device every compute call fails with MZH_ERR_HIP.
 */
#ifndef MZH_ABI_H_
#define MZH_ABI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MZH_ABI_VERSION 6

#define MZH_OK 0
#define MZH_ERR_ARG (-1)         /* bad argument / shape (ValueError in Python)              */
#define MZH_ERR_HIP (-2)         /* HIP runtime error / no device (RuntimeError)              */
#define MZH_ERR_CAPACITY (-3)    /* B > max_roots or n_sims > max_sims of the engine          */
#define MZH_ERR_STATE (-4)       /* weights not loaded                                        */
#define MZH_ERR_TEMPERATURE (-5) /* temperature outside [0,1] (mcts.py:163-166 ValueError)    */

#define MZH_ACTIONS 6   /* itertools.permutations(range(3), 2), env/hanoi.py:39-41 */
#define MZH_LATENT 64   /* reprs_output_size, networks.py:22 */
#define MZH_HIDDEN 256  /* h1_s, networks.py:21 */

/* search flags */
#define MZH_FLAG_NP1_UCB 1u /* UCB rounding of NumPy 1.x (the reference's pin, requirements.txt:17):
                               U = fl32(fl64(prior * w)); default is NumPy 2: fl32(prior * fl32(w)) */
#define MZH_FLAG_KERNEL_COOP 2u /* force the cooperative kernel (4 waves share one 32-root tile) */
#define MZH_FLAG_KERNEL_WAVE 4u /* force the wave-independent kernel, 32 roots per wave (default for B >= 53248) */
#define MZH_FLAG_KERNEL_WAVE16 8u /* force the wave-independent kernel, 16 roots per wave (default for 8192 < B < 53248) */
#define MZH_FLAG_COOP_TILE16 16u /* cooperative kernel: 16 roots per workgroup (default for B <= 4096) */
#define MZH_FLAG_COOP_TILE32 32u /* cooperative kernel: 32 roots per workgroup (default for B > 4096) */
#define MZH_FLAG_COOP_OCC2 64u /* cooperative kernel, 16-root tiles, two workgroups per CU
                                  (mzh_search_occ2_kernel).  An MLP search whose LDS does not fit twice per
                                  CU fails with MZH_ERR_CAPACITY; a replay (tree-only) search, which has no
                                  occ2 instantiation, runs the cooperative replay kernel instead (the plan
                                  names it) */
#define MZH_FLAG_KERNEL_ONE 128u /* force the latency kernel (mzh_search_one_kernel: one root per workgroup,
                                    the network stationary on the CU; default for MLP searches of B <= 512
                                    roots whose LDS fits).  An error for replay searches, with another kernel
                                    flag, or where its LDS does not fit */

typedef struct mzh_engine mzh_engine;
typedef void* mzh_stream; /* hipStream_t */

int mzh_abi_version(void);
const char* mzh_last_error(void);
/* Provenance: a hash of the csrc/ sources, include/mzh.h and the compiler flags this library was
 * built from (muzero-hanoi_amd/build.py source_hash); the Python binding refuses a library whose id
 * differs from the checked-out sources, and bench / smoke records print it. */
const char* mzh_build_id(void);
int mzh_device_count(int* count);
/* The device address of page-locked host memory (hipHostGetDevicePointer): the one-root drop-in calls
 * (MCTS.run_mcts, TowersOfHanoi.step) hand their few inputs and outputs to the kernels in pinned host memory
 * the kernels read and write directly, so a call is one launch and one synchronisation, no copies. */
int mzh_host_device_pointer(void* host, void** dev);
/* Wait for every call issued on `stream` (hipStreamSynchronize): the one-root drop-ins' single synchronisation
 * per call, without a framework stream object per call. */
int mzh_stream_synchronize(void* stream);

/* ---------------------------------------------------------------------------------------------
 * Engine.  Replaces the state the reference keeps in Python objects: the MuZeroNet weights
 * (networks.py:39-67) and the per-search node pool of MCTS/node.py (flat SoA tree workspace).
 *   n_disks   : Hanoi N (observation = 3N one-hot, env/hanoi.py:26-28, utils.py:9-25)
 *   max_sims  : largest n_simulations a search on this engine may use (mcts.py:30)
 *   max_roots : largest root batch B
 *   support   : 33 (TD_return=True) or 1 (TD_return=False), networks.py:34-37
 * ------------------------------------------------------------------------------------------- */
int mzh_create(int device, int n_disks, int max_sims, int max_roots, int support, mzh_engine** out);
int mzh_destroy(mzh_engine* eng);

/* Number of floats of the canonical flat weight vector: the 20 tensors of MuZeroNet.state_dict()
 * (networks.py:39-67) concatenated in the order
 *   {representation,dynamic,rwd,policy,value}_net.{0,2}.{weight,bias},
 * each in torch layout (nn.Linear weight [out][in] row-major). */
int mzh_weights_size(int n_disks, int support, size_t* n_floats);

/* Upload + repack (host pointer, canonical layout) into the MFMA fragment layout on the device.
 * Replaces reading MuZeroNet parameters at inference time (networks.py:71-150). Synchronous. */
int mzh_load_weights(mzh_engine* eng, const float* flat_host, size_t n_floats);

/* ---------------------------------------------------------------------------------------------
 * Environment: TowersOfHanoi (env/hanoi.py), batched over B independent envs.
 * state[B][n] uint8 peg of disc d (disc 0 = smallest), the reference's tuple c_state layout.
 * ------------------------------------------------------------------------------------------- */

/* TowersOfHanoi.step (env/hanoi.py:47-84) for every env b:
 *   state      in/out  c_state (unchanged on illegal moves and on the goal step, hanoi.py:65-74)
 *   action     in      index into moves = [(0,1),(0,2),(1,0),(1,2),(2,0),(2,1)]
 *   moved      out     state encoded by the returned observation (nullable)
 *   obs        out     oneHot_encoding(moved) as float32 [B][3n] (nullable; utils.py:9-25)
 *   reward     out     int8 code: 0 -> 0, 1 -> 100 (goal), -1 -> -100/1000 (illegal)
 *   done, illegal out  uint8
 *   step_ctr   in/out  step_counter (hanoi.py:50-80; illegal steps count, reset on done)
 *   active     in/out  reset_check (hanoi.py:49); stepping an inactive env is the reference's
 *                      AssertionError: the env is left untouched, reward = -2 and *err_count += 1
 *   err_count  out     nullable device int32 accumulator */
int mzh_env_step(int n_disks, int goal_peg, int max_steps, int B, uint8_t* state,
                 const int32_t* action, uint8_t* moved, float* obs, int8_t* reward, uint8_t* done,
                 uint8_t* illegal, int32_t* step_ctr, uint8_t* active, int32_t* err_count,
                 mzh_stream stream);

/* _move_allowed for all 6 moves (env/hanoi.py:117-139): bit a of mask[b] = move a legal. */
int mzh_legal_mask(int n_disks, int B, const uint8_t* state, uint8_t* mask, mzh_stream stream);

/* oneHot_encoding (utils.py:9-25): obs[b][3d + state[b][d]] = 1, float32. */
int mzh_encode_obs(int n_disks, int B, const uint8_t* state, float* obs, mzh_stream stream);

/* hanoi_solver (env/hanoi_utils.py:4-26): minimal moves to put every disc on goal_peg. */
int mzh_hanoi_solver(int n_disks, int goal_peg, int B, const uint8_t* state, int32_t* moves,
                     mzh_stream stream);

/* ---------------------------------------------------------------------------------------------
 * Network inference (MuZeroNet.initial_inference / recurrent_inference, networks.py:71-116),
 * batched over B rows.  Output pointers other than h may be NULL.
 *   h [B][64] normalised latent; reward [B] (0 for initial); pi [B][6] softmax policy;
 *   value [B] transformed value; *_logits raw head outputs ([B][6], [B][support]).
 * ------------------------------------------------------------------------------------------- */
int mzh_initial_inference(mzh_engine* eng, int B, const float* obs, float* h, float* reward,
                          float* pi, float* value, float* policy_logits, float* value_logits,
                          mzh_stream stream);
int mzh_recurrent_inference(mzh_engine* eng, int B, const float* h_in, const int32_t* action,
                            float* h, float* reward, float* pi, float* value,
                            float* policy_logits, float* value_logits, float* reward_logits,
                            mzh_stream stream);

/* ---------------------------------------------------------------------------------------------
 * Batched search: B independent MCTS.run_mcts calls (MCTS/mcts.py:34-126), one per root, all
 * simulations (select -> expand via the MLP -> backup) inside one fused kernel launch.
 * Each root carries its own MinMaxStats (utils_mcts.py): fresh unless minmax_in is given.
 * ------------------------------------------------------------------------------------------- */
typedef struct mzh_search_args {
  int32_t B;             /* roots */
  int32_t n_sims;        /* n_simulations (mcts.py:30) */
  double discount;       /* mcts.py:27 */
  double eps;            /* root_exploration_eps (mcts.py:20) */
  double temperature;    /* generate_play_policy temperature (mcts.py:154-176) */
  int32_t deterministic; /* argmax action instead of sampling (mcts.py:115-120) */
  uint32_t flags;        /* MZH_FLAG_* */
  /* inputs */
  const float* obs;         /* [B][3n] root observations (MLP mode) */
  const double* noise;      /* [B][6] Dirichlet draws, NULL = no noise (mcts.py:57-66) */
  const int32_t* tie_idx;   /* [B] pre-drawn index of np.random.choice for the first 6-way tie */
  const double* action_u;   /* [B] pre-drawn random_sample() for choice(6, p=pi); NULL if det. */
  const double* minmax_in;  /* [B][2] (maximum, minimum) or NULL (fresh: -inf, +inf) */
  /* replay (tree-only) inputs: network outputs recorded per simulation, used instead of the MLP
   * by mzh_search_replay */
  const float* rp_root_pi; /* [B][6] */
  const float* rp_sim;     /* [n_sims][B][8]: simulation s of root b = its 6 priors, reward, value --
                              simulation-major, so one simulation's reads of consecutive roots are
                              whole cache lines (32 B per root) */
  /* outputs (visits required, others nullable) */
  int32_t* visits;      /* [B][6] root child_N (node.py:133-136) */
  double* root_q;       /* [B] root_node.Q (node.py:125-131) */
  double* minmax_out;   /* [B][2] */
  int32_t* extra_ties;  /* [B] argmax ties beyond the first (RNG stream divergence indicator) */
  int32_t* action;      /* [B] chosen action (mcts.py:115-122) */
  double* pi;           /* [B][6] play policy (mcts.py:154-176) */
  int32_t* latent;      /* [B][n_sims+1] moves of the last simulation's path (mcts.py:79-86) */
  int32_t* latent_len;  /* [B] */
  int32_t* sel_steps;   /* [B] total selection steps (sum of depths), for byte accounting */
  /* play-policy power table (nullable): pow_table[n] = np.power(n, max(1, min(5, 1/T))) for
   * n = 0..n_sims as the caller's NumPy computes it (mcts.py:168-174).  Read only for a non-integer
   * exponent (integer exponents are exact products); without it the device pow is used, which can
   * differ from NumPy's vectorised pow in the last bit. */
  const double* pow_table;
  /* [lockstep groups] (nullable; entries of groups without roots are left untouched): per group of roots
   * that advance through a simulation together -- a wave of the wave kernel (16 or 32 roots, index
   * blockIdx * 4 + wave), a workgroup of the cooperative kernels, each root of the latency kernel (index =
   * root; so B entries cover every plan) -- the sum over simulations of the
   * group's deepest selection below the root, i.e. the dependent tree-block loads the group waits for in
   * sequence (the select / backup latency model, bench.py roofline.tree.latency) */
  int32_t* lockstep_levels;
  /* HOST pointer (nullable): filled with the plan of the launched instantiation (below); B = 0
   * launches nothing and reports kernel "none" */
  struct mzh_search_plan* plan_out;
} mzh_search_args;

/* What a search launch runs: the kernel instantiation chosen from B, n_sims, the flags, the
 * support and whether caller MinMaxStats bounds are given.  There is no reference counterpart (the
 * reference runs one Python MCTS per root, MCTS/mcts.py:34-126); it exists so measurements name
 * the kernel that actually ran. */
typedef struct mzh_search_plan {
  int32_t wave;                  /* 1: mzh_wave_kernel, 0: mzh_search_kernel (cooperative) */
  int32_t roots_per_wave;        /* wave: 16 or 32; cooperative: tile / 4 (tree-phase roots per wave) */
  int32_t roots_per_workgroup;   /* roots one workgroup owns */
  int32_t threads_per_workgroup;
  int32_t workgroups;            /* grid size */
  int64_t smem_bytes;            /* dynamic LDS per workgroup */
  char kernel[96];               /* the template instantiation as rocprofv3 names it, e.g.
                                    "mzh_search_kernel<32, false, true, true, false>" */
} mzh_search_plan;

int mzh_search(mzh_engine* eng, const mzh_search_args* args, mzh_stream stream);
int mzh_search_replay(mzh_engine* eng, const mzh_search_args* args, mzh_stream stream);
/* The plan mzh_search (replay = 0) / mzh_search_replay (replay = 1) would launch for these
 * arguments (has_minmax_in: args.minmax_in != NULL).  Host-only: needs no device and no engine. */
int mzh_search_plan_query(int support, int B, int n_sims, uint32_t flags, int replay, int has_minmax_in,
                          mzh_search_plan* out);

/* ---------------------------------------------------------------------------------------------
 * Reference-order host pre-draw (HOST pointers only; no device, no engine).  Replaces the NumPy
 * calls B sequential run_mcts calls make on the global legacy stream, in their order per call:
 *   np.random.dirichlet(np.ones_like(prob) * alpha)   MCTS/mcts.py:57-66,148-149  (k > 0)
 *   np.random.choice(<n_tie tied indices>)            MCTS/node.py:86             (n_tie > 1 draws)
 *   np.random.choice(np.arange(6), p=pi)              MCTS/mcts.py:118-120        (draw_action: the
 *                                                     one random_sample() it consumes)
 * NumPy's legacy RandomState algorithms (csrc/mzh_rng.cpp) on NumPy's own MT19937 state:
 *   mt_state    in/out  numpy mt19937_state {uint32 key[624]; int pos} (the bit generator's
 *                       ctypes.state_address), advanced in place exactly as NumPy would
 *   gauss_state in/out  {has_gauss, cached deviate} of the RandomState (read only for alpha > 1)
 *   alpha [k]           Dirichlet parameters as float64 (each > 0, else MZH_ERR_ARG as NumPy's
 *                       ValueError('alpha <= 0'))
 *   noise [B][k], tie [B] (index into the tied set), action_u [B]: outputs.
 * MZH_ERR_ARG for a bad argument, before anything is drawn. */
int mzh_rng_predraw(void* mt_state, double* gauss_state, int B, int k, const double* alpha, int n_tie,
                    int draw_action, double* noise, int32_t* tie, double* action_u);

/* ---------------------------------------------------------------------------------------------
 * Fused training update.  Replaces Muzero._update (Muzero.py:209-274: represent, U unrolled
 * prediction/dynamics steps, MSE value/reward and soft-target cross-entropy policy terms, the 0.5
 * latent-gradient hook, importance weights, the 1/U loss hook) and MuZeroNet.update's Adam step
 * (networks.py:69,118-122) for one sampled batch, in two kernel launches.
 *   B, U, in_dim, support : batch_s, unroll_n_steps, 3N, 33 (TD_return) or 1
 *   rows                  : transitions per workgroup of the row kernel (1 or 2; 0 = auto)
 *   step_size, bc2_sqrt   : torch.optim.Adam's lr / (1 - beta1^step) and sqrt(1 - beta2^step) for
 *                           this step (computed by the host in fp64, as torch does); beta1, beta2, eps
 *   obs [B][in_dim] f32, rwds [B][U] f32, actions [B][U] i64, pi [B][U][6] f32, returns [B][U] f32,
 *   weights [B] f32 importance weights or NULL (uniform replay)
 *   param / exp_avg / exp_avg_sq : the 20 MuZeroNet parameters in state_dict order
 *                           ({representation,dynamic,rwd,policy,value}_net.{0,2}.{weight,bias}) and
 *                           their Adam moments, updated in place
 *   wt[10]                : transposed copies [in][round_up(out, 4)] of the ten weights (param
 *                           0,2,...,18; pad columns zero), filled by mzh_train_transpose and kept
 *                           current by mzh_train_update
 *   scratch               : device workspace of mzh_train_scratch_bytes
 *   row_loss [B][3]       : per-transition value, reward and policy loss sums (their means are the
 *                           reference's returned losses); new_prio [B] = |v_0 - return_0| or NULL
 * ------------------------------------------------------------------------------------------- */
typedef struct mzh_train_args {
  int32_t B, U, in_dim, support, rows;
  float step_size, bc2_sqrt, beta1, beta2, eps;
  const float* obs;
  const float* rwds;
  const int64_t* actions;
  const float* pi;
  const float* returns;
  const float* weights;
  float* param[20];
  float* exp_avg[20];
  float* exp_avg_sq[20];
  float* wt[10];
  void* scratch;
  size_t scratch_bytes;
  float* row_loss;
  float* new_prio;
} mzh_train_args;

int mzh_train_scratch_bytes(int B, int U, int in_dim, int support, size_t* bytes);
int mzh_train_transpose(const mzh_train_args* args, mzh_stream stream);
int mzh_train_update(const mzh_train_args* args, mzh_stream stream);

/* ---------------------------------------------------------------------------------------------
 * Prioritised replay with the priorities resident in HBM, for the reference Buffer's defaults
 * (priority_exponent 1, importance_sampling_exponent 0: Muzero.py:72-78, buffer.py:13-14).
 *
 * mzh_replay_sample replaces Buffer.priority_sample's draw and batch (buffer.py:89-112): P = p / np.sum(p)
 * in float32, np.random.choice(np.arange(n), m, replace=True, p=P) from the uniforms u as RandomState
 * computes it (float64 cdf, cdf /= cdf[-1], searchsorted(u, side='right')), then the sampled rows.  The
 * indices equal NumPy's for the same u (np.random.random_sample(m), drawn by the caller).  One workgroup.
 *   n, m             : len(buffer) and batch_s (n >= 1, m >= 1)
 *   d_state, U, A    : row widths of the five transition arrays (states [.][d_state], rwds / returns
 *                      [.][U], actions int64 [.][U], pi [.][U][A])
 *   prio [n]         : device priorities (16-byte aligned)
 *   u [m]            : uniforms, device-readable (device or mapped page-locked memory)
 *   cdf [n]          : float64 workspace (the kernel keeps the cdf at every 4th element)
 *   indx [m]         : sampled indices (out)
 *   out_* [m][.]     : the sampled rows (out)
 *   status [2]       : device-written (out): [0] 0 = drawn, 1 = P has a NaN or negative entry (NumPy
 *                      raises ValueError there; indices and rows are then 0 / row 0); [1] 1 = the cdf
 *                      came from the exact parallel scan, 0 = from the sequential chain
 * mzh_replay_set_priorities replaces Buffer.update_priorities (buffer.py:127-134): prio[indx[k]] = values[k]
 * for k = 0..m-1, the last of repeated indices winning as in NumPy's fancy assignment, unless the
 * reference's assertion (all values finite, one > 0) fails or an index is outside [0, size): then nothing
 * is written and status[0] = 1 (assertion) / 2 (index), else 0.
 * ------------------------------------------------------------------------------------------- */
typedef struct mzh_replay_args {
  int32_t n, m, d_state, U, A;
  const float* prio;
  const double* u;
  double* cdf;
  const float* states;
  const float* rwds;
  const int64_t* actions;
  const float* pi;
  const float* returns;
  int64_t* indx;
  float* out_states;
  float* out_rwds;
  int64_t* out_actions;
  float* out_pi;
  float* out_returns;
  int32_t* status;
} mzh_replay_args;

int mzh_replay_sample(const mzh_replay_args* args, mzh_stream stream);
int mzh_replay_set_priorities(float* prio, int64_t size, const int64_t* indx, const float* values, int m,
                              int32_t* status, mzh_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* MZH_ABI_H_ */
