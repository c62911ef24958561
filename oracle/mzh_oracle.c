/*
 * mzh_oracle.c -- CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the CHECKER.  The product path (muzero-hanoi_amd/, libmzh.so) never links,
 * loads or falls back to it.
 *
 * Parity pinning: checked against the tests/golden fixtures, which tests/golden/gen_golden.py produced
 * by running the reference (A-Andrews/Muzero-Hanoi) itself in the build container:
 *   env tables (exhaustive, bit-exact), hanoi_solver KATs, MLP logits (<=1e-5 vs torch-CPU),
 *   replayed run_mcts traces (visit counts / pi / rootQ / min-max bit-exact).
 *
 * Every function cites the reference lines it restates.  Floating-point rules (build with
 * -O2 -ffp-contract=off, never -ffast-math):
 *   - tree statistics are fp64 in the reference's Python operation order (MCTS/node.py);
 *   - the MLP is fp32 with each dot product a k-ordered fmaf chain starting at 0, bias added
 *     after (the order a gfx950 f32 MFMA produces), softmax with mzh_expf (below) -- torch-CPU's
 *     own GEMV/exp/sqrt orders are not reproducible, so logits agree with torch at ~1e-7 while
 *     the transformed value/reward can move by up to ~1.4e-3.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_A 6     /* actions: permutations(range(3),2), env/hanoi.py:39-41 */
#define ORC_H 64    /* reprs_output_size, networks.py:22 */
#define ORC_F 256   /* h1_s, networks.py:21 */
#define ORC_MAXSUP 33

/* ------------------------------------------------------------------------------------------ */
/* Environment: env/hanoi.py                                                                  */
/* ------------------------------------------------------------------------------------------ */
static const int MOVES[6][2] = {{0, 1}, {0, 2}, {1, 0}, {1, 2}, {2, 0}, {2, 1}}; /* hanoi.py:39-41 */

/* _discs_on_peg + _move_allowed (env/hanoi.py:117-139): peg f non-empty and (t empty or
 * min(t) > min(f)). Restated literally with the two disc lists' minima. */
static int move_allowed(int n, const uint8_t* st, int f, int t) {
  int min_f = -1, min_t = -1;
  for (int d = 0; d < n; ++d) {
    if (st[d] == f && min_f < 0) min_f = d;
    if (st[d] == t && min_t < 0) min_t = d;
  }
  if (min_f < 0) return 0;
  if (min_t < 0) return 1;
  return min_t > min_f;
}

int orc_legal_mask(int n, const uint8_t* state) {
  int m = 0;
  for (int a = 0; a < ORC_A; ++a) m |= move_allowed(n, state, MOVES[a][0], MOVES[a][1]) << a;
  return m;
}

/* TowersOfHanoi.step (env/hanoi.py:47-84) for one env.
 *   state[n]     in/out: c_state (NOT advanced on the goal step, hanoi.py:65-69)
 *   moved[n]     out: the state the returned one-hot encodes
 *   *ctr         in/out: step_counter; *active in/out: reset_check
 *   returns reward code: 0 -> 0, 1 -> 100 (goal), -1 -> -100/1000 (illegal); -2 = step before reset */
int orc_env_step(int n, int goal_peg, int max_steps, uint8_t* state, int action, uint8_t* moved,
                 int* ctr, uint8_t* active, uint8_t* done, uint8_t* illegal) {
  if (!*active) return -2; /* assert self.reset_check, hanoi.py:49 */
  int f = MOVES[action][0], t = MOVES[action][1];
  int ill = !move_allowed(n, state, f, t);
  int code;
  *ctr += 1;
  memcpy(moved, state, (size_t)n);
  *done = 0;
  if (!ill) {
    int disc = -1;
    for (int d = 0; d < n; ++d)
      if (state[d] == f) { disc = d; break; } /* min(discs_on_peg(f)), hanoi.py:141-151 */
    moved[disc] = (uint8_t)t;
    int is_goal = 1;
    for (int d = 0; d < n; ++d) is_goal &= (moved[d] == goal_peg);
    if (!is_goal) {
      code = 0;
      memcpy(state, moved, (size_t)n);
    } else {
      code = 1;
      *done = 1;
      *active = 0;
      *ctr = 0;
    }
  } else {
    code = -1; /* rwd = -100/1000, state unchanged */
  }
  if (*ctr == max_steps) { /* hanoi.py:77-80 */
    *done = 1;
    *active = 0;
    *ctr = 0;
  }
  *illegal = (uint8_t)ill;
  return code;
}

/* hanoi_solver (env/hanoi_utils.py:4-26) */
long orc_hanoi_solver(int n, const uint8_t* state, int goal_peg) {
  long moves = 0;
  int target = goal_peg;
  for (int i = n - 1; i >= 0; --i) {
    if (state[i] != target) {
      moves += 1L << i;
      target = 3 - target - state[i];
    }
  }
  return moves;
}

/* ------------------------------------------------------------------------------------------ */
/* fp32 math restatement (networks.py:152-196)                                                */
/* ------------------------------------------------------------------------------------------ */
/* Deterministic expf (Cody-Waite reduction + degree-6 polynomial, explicit fmaf). The same
 * algorithm is implemented on the device (mzh_device.h), so both sides produce identical bits. */
float orc_expf(float x) {
  if (x < -87.0f) return 0.0f;
  if (x > 88.0f) return INFINITY;
  float n = rintf(x * 1.44269502162933349609375f);
  float r = fmaf(n, -0.693359375f, x);
  r = fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = fmaf(p, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  p = fmaf(p, r2, r);
  p = p + 1.0f;
  int ni = (int)n;
  union { uint32_t u; float f; } s;
  s.u = (uint32_t)(ni + 127) << 23;
  return p * s.f;
}

/* Fixed summation order shared with the device (8 lanes, one partial sum each):
 *   s_q = v[q] + v[q+8] + v[q+16] + ...  (sequential, q = 0..7; 0 when q >= n)
 *   sum = ((s_0 + s_1) + (s_2 + s_3)) + ((s_4 + s_5) + (s_6 + s_7))
 * torch's own reduction order for these sums is an implementation detail of its vectorised
 * kernels; any fixed order is an equally faithful restatement (within the tolerances of
 * SURVEY.md 8a-10), and this one maps onto an 8-lane DPP tree. */
static float sum8_tree(const float* v, int n) {
  float s[8];
  for (int q = 0; q < 8; ++q) {
    float a = 0.0f;
    if (q < n) {
      a = v[q];
      for (int k = q + 8; k < n; k += 8) a = a + v[k];
    }
    s[q] = a;
  }
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

/* F.softmax over the last dim (networks.py:83,109,170) */
static void softmax(const float* l, int n, float* p) {
  float m = l[0];
  for (int i = 1; i < n; ++i)
    if (l[i] > m) m = l[i];
  for (int i = 0; i < n; ++i) p[i] = orc_expf(l[i] - m);
  const float s = sum8_tree(p, n);
  for (int i = 0; i < n; ++i) p[i] = p[i] / s;
}

/* _signed_parabolic (networks.py:186-189), python scalars folded in fp64 then rounded to fp32:
 * eps+1 -> 1.001f, 4*eps -> 0.004f, /eps -> /0.001f, 1/2/eps -> 500. */
float orc_signed_parabolic(float x) {
  float a = fabsf(x);
  float t = 1.00100004673004150390625f + a;
  t = 0.0040000001899898052215576171875f * t;
  t = 1.0f + t;
  t = sqrtf(t);
  t = t / 2.0f;
  t = t / 0.001000000047497451305389404296875f;
  float z = t - 500.0f;
  float sg = x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f);
  return sg * (z * z - 1.0f);
}

/* logits_to_transformed_expected_value (networks.py:152-184): softmax, sum p_k * support_k
 * (support = linspace(-16,16,33), exact integers), then _signed_parabolic. */
float orc_logits_to_value(const float* logits, int support) {
  if (support == 1) return logits[0]; /* TD_return=False: no transform, networks.py:146-148 */
  float p[ORC_MAXSUP];
  softmax(logits, support, p);
  int half = (support - 1) / 2;
  float prod[ORC_MAXSUP];
  for (int k = 0; k < support; ++k) prod[k] = p[k] * (float)(k - half);
  return orc_signed_parabolic(sum8_tree(prod, support));
}

/* the expected scalar before the transform (networks.py:174-184: softmax, sum p_k * support_k) --
 * the argument orc_logits_to_value hands to orc_signed_parabolic (test attribution only) */
float orc_logits_expectation(const float* logits, int support) {
  if (support == 1) return logits[0];
  float p[ORC_MAXSUP];
  softmax(logits, support, p);
  int half = (support - 1) / 2;
  float prod[ORC_MAXSUP];
  for (int k = 0; k < support; ++k) prod[k] = p[k] * (float)(k - half);
  return sum8_tree(prod, support);
}

/* normalize_h_state (networks.py:191-196) */
static void normalize_h(float* h) {
  float mn = h[0], mx = h[0];
  for (int i = 1; i < ORC_H; ++i) {
    if (h[i] < mn) mn = h[i];
    if (h[i] > mx) mx = h[i];
  }
  float d = (mx - mn) + 9.999999939225290290778502821922302246094e-09f;
  for (int i = 0; i < ORC_H; ++i) h[i] = (h[i] - mn) / d;
}

/* ------------------------------------------------------------------------------------------ */
/* MLP (networks.py:39-67, 71-150).  Weights: the canonical flat layout of include/mzh.h --    */
/* the 20 state_dict tensors concatenated in key order, each in torch layout [out][in].       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int in_dim, support;
  const float *rep0_w, *rep0_b, *rep2_w, *rep2_b;
  const float *dyn0_w, *dyn0_b, *dyn2_w, *dyn2_b;
  const float *rwd0_w, *rwd0_b, *rwd2_w, *rwd2_b;
  const float *pol0_w, *pol0_b, *pol2_w, *pol2_b;
  const float *val0_w, *val0_b, *val2_w, *val2_b;
} orc_weights;

size_t orc_weights_size(int in_dim, int support) {
  size_t s = 0;
  s += (size_t)ORC_F * in_dim + ORC_F + (size_t)ORC_H * ORC_F + ORC_H;            /* rep */
  s += (size_t)ORC_F * (ORC_H + ORC_A) + ORC_F + (size_t)ORC_H * ORC_F + ORC_H;   /* dyn */
  s += (size_t)ORC_F * ORC_H + ORC_F + (size_t)support * ORC_F + support;         /* rwd */
  s += (size_t)ORC_F * ORC_H + ORC_F + (size_t)ORC_A * ORC_F + ORC_A;             /* policy */
  s += (size_t)ORC_F * ORC_H + ORC_F + (size_t)support * ORC_F + support;         /* value */
  return s;
}

static void bind_weights(orc_weights* w, const float* flat, int in_dim, int support) {
  const float* p = flat;
#define TAKE(field, cnt) do { w->field = p; p += (cnt); } while (0)
  w->in_dim = in_dim;
  w->support = support;
  TAKE(rep0_w, ORC_F * in_dim); TAKE(rep0_b, ORC_F); TAKE(rep2_w, ORC_H * ORC_F); TAKE(rep2_b, ORC_H);
  TAKE(dyn0_w, ORC_F * (ORC_H + ORC_A)); TAKE(dyn0_b, ORC_F); TAKE(dyn2_w, ORC_H * ORC_F); TAKE(dyn2_b, ORC_H);
  TAKE(rwd0_w, ORC_F * ORC_H); TAKE(rwd0_b, ORC_F); TAKE(rwd2_w, support * ORC_F); TAKE(rwd2_b, support);
  TAKE(pol0_w, ORC_F * ORC_H); TAKE(pol0_b, ORC_F); TAKE(pol2_w, ORC_A * ORC_F); TAKE(pol2_b, ORC_A);
  TAKE(val0_w, ORC_F * ORC_H); TAKE(val0_b, ORC_F); TAKE(val2_w, support * ORC_F); TAKE(val2_b, support);
#undef TAKE
}

/* nn.Linear with a k-ordered fmaf chain from 0, bias after, optional ReLU */
static void linear(const float* x, int K, const float* W, const float* b, int N, float* y, int relu) {
  for (int n = 0; n < N; ++n) {
    const float* wr = W + (size_t)n * K;
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) acc = fmaf(x[k], wr[k], acc);
    float v = acc + b[n];
    if (relu) v = v > 0.0f ? v : 0.0f;
    y[n] = v;
  }
}

/* The value / reward output layer (33 support bins): bins 0..31 as `linear` (the GPU's MFMA tiles),
 * bin 32 -- the one logit past two 16-row tiles -- as four k-ordered fmaf chains over k = g, g + 4,
 * g + 8, ... (g = 0..3) combined ((p0 + p1) + (p2 + p3)), bias after: the order the GPU kernels
 * compute it in with vector FMAs instead of a third, 15/16-padding MFMA tile (muzero-hanoi_amd/csrc,
 * MzhWMlp::w32) */
static void linear_head(const float* x, const float* W, const float* b, int N, float* y) {
  if (N != ORC_MAXSUP) {
    linear(x, ORC_F, W, b, N, y, 0);
    return;
  }
  linear(x, ORC_F, W, b, N - 1, y, 0);
  const float* wr = W + (size_t)(N - 1) * ORC_F;
  float p[4];
  for (int g = 0; g < 4; ++g) {
    float acc = 0.0f;
    for (int k = g; k < ORC_F; k += 4) acc = fmaf(x[k], wr[k], acc);
    p[g] = acc;
  }
  y[N - 1] = ((p[0] + p[1]) + (p[2] + p[3])) + b[N - 1];
}

typedef struct {
  float h[ORC_H];
  float reward;
  float pi[ORC_A];
  float value;
  float policy_logits[ORC_A];
  float value_logits[ORC_MAXSUP];
  float reward_logits[ORC_MAXSUP];
} orc_netout;

/* prediction (networks.py:140-150) + softmax of the policy logits */
static void prediction(const orc_weights* w, const float* h, orc_netout* o) {
  float hid[ORC_F];
  linear(h, ORC_H, w->pol0_w, w->pol0_b, ORC_F, hid, 1);
  linear(hid, ORC_F, w->pol2_w, w->pol2_b, ORC_A, o->policy_logits, 0);
  linear(h, ORC_H, w->val0_w, w->val0_b, ORC_F, hid, 1);
  linear_head(hid, w->val2_w, w->val2_b, w->support, o->value_logits);
  o->value = orc_logits_to_value(o->value_logits, w->support);
  softmax(o->policy_logits, ORC_A, o->pi);
}

/* initial_inference (networks.py:71-94): h = norm(rep(x)), rwd := 0 */
static void initial_inference(const orc_weights* w, const float* x, orc_netout* o) {
  float hid[ORC_F];
  linear(x, w->in_dim, w->rep0_w, w->rep0_b, ORC_F, hid, 1);
  linear(hid, ORC_F, w->rep2_w, w->rep2_b, ORC_H, o->h, 0);
  normalize_h(o->h);
  prediction(w, o->h, o);
  o->reward = 0.0f;
  memset(o->reward_logits, 0, sizeof(o->reward_logits));
}

/* recurrent_inference (networks.py:96-138): x = cat(h, onehot(a)); h' = dyn(x);
 * reward from h' (un-normalised); h = norm(h'); prediction(h) */
static void recurrent_inference(const orc_weights* w, const float* h_in, int action, orc_netout* o) {
  float x[ORC_H + ORC_A];
  float hid[ORC_F];
  memcpy(x, h_in, sizeof(float) * ORC_H);
  for (int a = 0; a < ORC_A; ++a) x[ORC_H + a] = (a == action) ? 1.0f : 0.0f;
  linear(x, ORC_H + ORC_A, w->dyn0_w, w->dyn0_b, ORC_F, hid, 1);
  linear(hid, ORC_F, w->dyn2_w, w->dyn2_b, ORC_H, o->h, 0);
  linear(o->h, ORC_H, w->rwd0_w, w->rwd0_b, ORC_F, hid, 1);
  linear_head(hid, w->rwd2_w, w->rwd2_b, w->support, o->reward_logits);
  o->reward = orc_logits_to_value(o->reward_logits, w->support);
  normalize_h(o->h);
  prediction(w, o->h, o);
}

/* Batched MLP entry points (row loop; rows independent). Output pointers may be NULL. */
void orc_initial_inference(const float* flat, int in_dim, int support, int B, const float* x,
                           float* h, float* reward, float* pi, float* value,
                           float* policy_logits, float* value_logits) {
  orc_weights w;
  bind_weights(&w, flat, in_dim, support);
  for (int b = 0; b < B; ++b) {
    orc_netout o;
    initial_inference(&w, x + (size_t)b * in_dim, &o);
    if (h) memcpy(h + (size_t)b * ORC_H, o.h, sizeof(o.h));
    if (reward) reward[b] = o.reward;
    if (pi) memcpy(pi + (size_t)b * ORC_A, o.pi, sizeof(o.pi));
    if (value) value[b] = o.value;
    if (policy_logits) memcpy(policy_logits + (size_t)b * ORC_A, o.policy_logits, sizeof(o.policy_logits));
    if (value_logits) memcpy(value_logits + (size_t)b * support, o.value_logits, sizeof(float) * support);
  }
}

void orc_recurrent_inference(const float* flat, int in_dim, int support, int B, const float* h_in,
                             const int* action, float* h, float* reward, float* pi, float* value,
                             float* policy_logits, float* value_logits, float* reward_logits) {
  orc_weights w;
  bind_weights(&w, flat, in_dim, support);
  for (int b = 0; b < B; ++b) {
    orc_netout o;
    recurrent_inference(&w, h_in + (size_t)b * ORC_H, action[b], &o);
    if (h) memcpy(h + (size_t)b * ORC_H, o.h, sizeof(o.h));
    if (reward) reward[b] = o.reward;
    if (pi) memcpy(pi + (size_t)b * ORC_A, o.pi, sizeof(o.pi));
    if (value) value[b] = o.value;
    if (policy_logits) memcpy(policy_logits + (size_t)b * ORC_A, o.policy_logits, sizeof(o.policy_logits));
    if (value_logits) memcpy(value_logits + (size_t)b * support, o.value_logits, sizeof(float) * support);
    if (reward_logits) memcpy(reward_logits + (size_t)b * support, o.reward_logits, sizeof(float) * support);
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Search: MCTS/mcts.py:34-176, MCTS/node.py:6-136, MCTS/utils_mcts.py:1-16                   */
/* ------------------------------------------------------------------------------------------ */
#define PB_C_BASE 19652 /* mcts.py:24 */
#define PB_C_INIT 1.25  /* mcts.py:25 */

/* (log((N + base + 1) / base) + init) * sqrt(N)   -- node.py:114-121 up to the "/ (child.N+1)" */
/* Property check for the device's division (csrc/mzh_search.hip mzh_div): a / b computed as
 * q = a*y, r = fma(-q, b, a), q' = fma(r, y, q) with y = RN(1/b) must equal IEEE a / b.  Runs n
 * random trials over the select/backup operand domains (W / N and table[Np] / (N + 1) with integer
 * N in [1, 64]; normalise's (v - min) / (max - min) with real denominators) and returns the number
 * of mismatches (test infrastructure only, not part of the reference algorithm). */
static uint64_t mk_s;
static uint64_t mk_next(void) {
  mk_s ^= mk_s << 13;
  mk_s ^= mk_s >> 7;
  mk_s ^= mk_s << 17;
  return mk_s;
}
static double mk_unit(void) { return (double)(mk_next() >> 11) * (1.0 / 9007199254740992.0); }
static double mk_rand_exp(int lo, int span) {
  uint64_t u = mk_next();
  u &= ~(0xfffull << 52);
  u |= ((uint64_t)(1023 + lo + (int)(mk_next() % (uint64_t)span))) << 52;
  double d;
  memcpy(&d, &u, 8);
  return d;
}
long orc_markstein_mismatches(long n, uint64_t seed) {
  long bad = 0;
  mk_s = seed ? seed : 88172645463325252ull;
  for (long i = 0; i < n; ++i) {
    double a, b;
    if (i & 1) {
      b = (double)(1 + (int)(mk_next() % 64));
      switch (mk_next() % 3) {
        case 0: a = (mk_unit() * 2 - 1) * 200.0; break;
        case 1: a = ldexp(mk_unit() * 2 - 1, (int)(mk_next() % 60) - 30); break;
        default: a = mk_rand_exp(-20, 40); break;
      }
    } else {
      b = (mk_next() & 1) ? mk_unit() * 10 + 1e-9 : mk_rand_exp(-15, 30);
      a = (mk_next() & 1) ? (mk_unit() * 2 - 1) * ldexp(1.0, (int)(mk_next() % 20) - 10) : mk_rand_exp(-15, 30);
    }
    const double y = 1.0 / b;
    const double q = a * y;
    const double r = fma(-q, b, a);
    if (fma(r, y, q) != a / b) ++bad;
  }
  return bad;
}

double orc_ucb_table(int n) {
  return (log((double)(n + PB_C_BASE + 1) / (double)PB_C_BASE) + PB_C_INIT) * sqrt((double)n);
}

typedef struct {
  int N;
  double W;
  double rwd;        /* python float: the fp32 network reward widened */
  double prior64;    /* prior value (exact) */
  int prior_is_f64;  /* root children after Dirichlet mixing are np.float64 (mcts.py:150) */
  int first_child;   /* -1 = not expanded */
  int parent;
  int move;
  int hslot;         /* index of this node's latent in the latent buffer, -1 if none */
} orc_node;

typedef struct {
  double maximum, minimum; /* MinMaxStats (utils_mcts.py:1-16): max=-inf, min=+inf */
} orc_minmax;

static void mm_update(orc_minmax* m, double v) {
  if (v > m->maximum) m->maximum = v; /* python max(self.maximum, value) */
  if (v < m->minimum) m->minimum = v;
}
static double mm_normalize(const orc_minmax* m, double v) {
  if (m->maximum > m->minimum) return (v - m->minimum) / (m->maximum - m->minimum);
  return v;
}

enum { ORC_FLAG_NP1_UCB = 1 };

typedef struct {
  /* network: either weights (MLP mode) or recorded outputs (replay mode) */
  const orc_weights* w;
  const float* rp_root_pi; /* [6] */
  const float* rp_pi;      /* [S][6] */
  const float* rp_rwd;     /* [S] */
  const float* rp_val;     /* [S] */
} orc_net;

/* One run_mcts for one root (MCTS/mcts.py:34-126). */
static void search_one(int S, double discount, int flags, const orc_net* net, const float* obs,
                       const double* noise, double eps, int tie_idx, const double* table,
                       orc_minmax* mm, orc_node* nodes, float* hbuf, int* visits, double* rootQ,
                       int* extra_ties, int* latent, int* latent_len, long* sel_steps, int* depths) {
  int n_nodes = 0;
  int n_h = 0;
  float root_pi[ORC_A];
  /* root: initial_inference (mcts.py:49-50) */
  if (net->w) {
    orc_netout o;
    initial_inference(net->w, obs, &o);
    memcpy(hbuf, o.h, sizeof(o.h));
    memcpy(root_pi, o.pi, sizeof(root_pi));
  } else {
    memcpy(root_pi, net->rp_root_pi, sizeof(root_pi));
  }
  n_h = 1;
  orc_node* root = &nodes[n_nodes++];
  root->N = 0; root->W = 0.0; root->rwd = 0.0; root->prior64 = 0.0; root->prior_is_f64 = 0;
  root->parent = -1; root->move = -1; root->hslot = 0;
  /* root.expand(prior, h, rwd) with optional Dirichlet mixing (mcts.py:57-69, 132-152) */
  root->first_child = n_nodes;
  for (int a = 0; a < ORC_A; ++a) {
    orc_node* c = &nodes[n_nodes++];
    c->N = 0; c->W = 0.0; c->rwd = 0.0; c->first_child = -1; c->parent = 0; c->move = a; c->hslot = -1;
    if (noise) {
      /* (1 - eps) * prob [float32 array, python scalar cast to f32] + eps * noise [f64] */
      float scaled = (float)(1.0 - eps) * root_pi[a];
      c->prior64 = (double)scaled + eps * noise[a];
      c->prior_is_f64 = 1;
    } else {
      c->prior64 = (double)root_pi[a];
      c->prior_is_f64 = 0;
    }
  }
  int first_tie_used = 0;
  *extra_ties = 0;
  long steps = 0;
  for (int s = 0; s < S; ++s) {
    /* Phase 1: select (mcts.py:75-86, node.py:72-123) */
    int node = 0;
    int depth = 0;
    while (nodes[node].first_child >= 0) {
      orc_node* p = &nodes[node];
      float ucb[ORC_A];
      for (int a = 0; a < ORC_A; ++a) {
        orc_node* c = &nodes[p->first_child + a];
        float q32;
        if (c->N > 0)
          q32 = (float)mm_normalize(mm, c->rwd + discount * (c->W / (double)c->N));
        else
          q32 = 0.0f;
        double w = table[p->N] / (double)(c->N + 1);
        float u32;
        if (c->prior_is_f64 || (flags & ORC_FLAG_NP1_UCB))
          u32 = (float)(c->prior64 * w);                 /* fl32(fl64(prior * w)) */
        else
          u32 = (float)c->prior64 * (float)w;            /* NumPy-2: fl32(prior32 * fl32(w)) */
        ucb[a] = q32 + u32;
      }
      float mx = ucb[0];
      for (int a = 1; a < ORC_A; ++a)
        if (ucb[a] > mx) mx = ucb[a];
      int cand[ORC_A], nc = 0;
      for (int a = 0; a < ORC_A; ++a)
        if (ucb[a] == mx) cand[nc++] = a;
      int pick;
      if (nc == 1) {
        pick = cand[0];
      } else if (!first_tie_used && nc == ORC_A) {
        pick = cand[tie_idx]; /* np.random.choice(argmax set): the host pre-drew this index */
        first_tie_used = 1;
      } else {
        pick = cand[0];
        *extra_ties += 1;
      }
      node = p->first_child + pick;
      if (latent && s == S - 1) latent[depth] = pick;
      depth++;
      steps++;
    }
    if (latent_len && s == S - 1) *latent_len = depth;
    if (depths) depths[s] = depth; /* this simulation's selection depth (levels below the root + 1) */
    /* Phase 2: expand leaf from parent's latent and the leaf's move (mcts.py:88-106) */
    orc_node* leaf = &nodes[node];
    orc_node* par = &nodes[leaf->parent];
    float pi[ORC_A];
    double value, reward;
    if (net->w) {
      orc_netout o;
      recurrent_inference(net->w, hbuf + (size_t)par->hslot * ORC_H, leaf->move, &o);
      memcpy(hbuf + (size_t)n_h * ORC_H, o.h, sizeof(o.h));
      memcpy(pi, o.pi, sizeof(pi));
      value = (double)o.value;
      reward = (double)o.reward;
    } else {
      memcpy(pi, net->rp_pi + (size_t)s * ORC_A, sizeof(pi));
      value = (double)net->rp_val[s];
      reward = (double)net->rp_rwd[s];
    }
    leaf->hslot = n_h++;
    leaf->rwd = reward;
    leaf->first_child = n_nodes;
    for (int a = 0; a < ORC_A; ++a) {
      orc_node* c = &nodes[n_nodes++];
      c->N = 0; c->W = 0.0; c->rwd = 0.0; c->first_child = -1; c->parent = node; c->move = a;
      c->hslot = -1; c->prior64 = (double)pi[a]; c->prior_is_f64 = 0;
    }
    /* Phase 3: backup (node.py:53-70) */
    int cur = node;
    while (cur >= 0) {
      orc_node* c = &nodes[cur];
      c->W += value;
      c->N += 1;
      mm_update(mm, c->rwd + discount * (c->W / (double)c->N));
      value = c->rwd + discount * value;
      cur = c->parent;
    }
  }
  orc_node* r = &nodes[0];
  for (int a = 0; a < ORC_A; ++a) visits[a] = nodes[r->first_child + a].N;
  *rootQ = r->N == 0 ? 0.0 : r->W / (double)r->N; /* node.py:125-131 */
  if (sel_steps) *sel_steps = steps;
}

/* generate_play_policy + action choice (mcts.py:111-122, 154-176) and legacy
 * RandomState.choice(6, p=pi): cdf = cumsum(p); cdf /= cdf[-1]; searchsorted(u, 'right').
 * powtab (nullable): powtab[n] = np.power(n, e) as the caller's NumPy computes it (mcts.py:174);
 * used for a non-integer exponent, where NumPy's vectorised pow (SVML on AVX-512 hosts) and libm's
 * pow differ in the last bit for some n.  Integer exponents are exact products either way.
 * Returns -1 on an invalid temperature (ValueError). */
int orc_play_policy(const int* visits, double temperature, int deterministic, double u, const double* powtab,
                    double* pi) {
  if (!(temperature >= 0.0 && temperature <= 1.0)) return -1;
  double v[ORC_A];
  for (int a = 0; a < ORC_A; ++a) v[a] = (double)visits[a];
  if (temperature > 0.0) {
    double e = 1.0 / temperature;
    if (e > 5.0) e = 5.0;
    if (e < 1.0) e = 1.0;
    const int integral = e == rint(e);
    for (int a = 0; a < ORC_A; ++a) v[a] = (powtab && !integral) ? powtab[visits[a]] : pow(v[a], e);
  }
  double sum = 0.0;
  for (int a = 0; a < ORC_A; ++a) sum += v[a];
  for (int a = 0; a < ORC_A; ++a) pi[a] = v[a] / sum;
  if (deterministic) {
    int best = 0;
    for (int a = 1; a < ORC_A; ++a)
      if (visits[a] > visits[best]) best = a;
    return best;
  }
  double cdf[ORC_A];
  double c = 0.0;
  for (int a = 0; a < ORC_A; ++a) {
    c += pi[a];
    cdf[a] = c;
  }
  double last = cdf[ORC_A - 1];
  for (int a = 0; a < ORC_A; ++a) cdf[a] = cdf[a] / last;
  for (int a = 0; a < ORC_A; ++a)
    if (cdf[a] > u) return a;
  return ORC_A; /* u >= 1: not reachable for random_sample() in [0,1) */
}

/* Batched search: B independent roots, each a fresh (or given) MinMaxStats.
 * Network = MLP (flat != NULL) or replay (rp_* != NULL).  All output pointers may be NULL
 * except visits.  depths [B][S] (nullable): every simulation's selection depth, the input of the
 * lockstep-grouping price (tools/price_grouping.py). */
int orc_search(int n_disks, int S, int B, double discount, int flags, const float* flat,
               int support, const float* obs, const float* rp_root_pi, const float* rp_pi,
               const float* rp_rwd, const float* rp_val, const double* noise, double eps,
               const int* tie_idx, const double* action_u, double temperature, int deterministic,
               const double* powtab, const double* minmax_in, int* visits, double* rootQ, double* minmax_out,
               int* extra_ties, int* action, double* pi, int* latent, int* latent_len,
               long* sel_steps, int* depths) {
  int in_dim = 3 * n_disks;
  orc_weights w;
  if (flat) bind_weights(&w, flat, in_dim, support);
  double* table = (double*)malloc(sizeof(double) * (size_t)(S + 2));
  orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (size_t)(6 * S + 7));
  float* hbuf = (float*)malloc(sizeof(float) * (size_t)(S + 1) * ORC_H);
  if (!table || !nodes || !hbuf) { free(table); free(nodes); free(hbuf); return -1; }
  for (int i = 0; i <= S + 1; ++i) table[i] = orc_ucb_table(i);
  int status = 0;
  for (int b = 0; b < B; ++b) {
    orc_net net;
    memset(&net, 0, sizeof(net));
    if (flat) {
      net.w = &w;
    } else {
      net.rp_root_pi = rp_root_pi + (size_t)b * ORC_A;
      net.rp_pi = rp_pi + (size_t)b * S * ORC_A;
      net.rp_rwd = rp_rwd + (size_t)b * S;
      net.rp_val = rp_val + (size_t)b * S;
    }
    orc_minmax mm = {-INFINITY, INFINITY};
    if (minmax_in) { mm.maximum = minmax_in[2 * b]; mm.minimum = minmax_in[2 * b + 1]; }
    int et = 0, ll = 0;
    long st = 0;
    double q;
    search_one(S, discount, flags, &net, obs + (size_t)b * in_dim, noise ? noise + (size_t)b * ORC_A : NULL,
               eps, tie_idx ? tie_idx[b] : 0, table, &mm, nodes, hbuf, visits + (size_t)b * ORC_A, &q, &et,
               latent ? latent + (size_t)b * (S + 1) : NULL, &ll, &st, depths ? depths + (size_t)b * S : NULL);
    if (rootQ) rootQ[b] = q;
    if (minmax_out) { minmax_out[2 * b] = mm.maximum; minmax_out[2 * b + 1] = mm.minimum; }
    if (extra_ties) extra_ties[b] = et;
    if (latent_len) latent_len[b] = ll;
    if (sel_steps) sel_steps[b] = st;
    if (action || pi) {
      double p[ORC_A];
      int act = orc_play_policy(visits + (size_t)b * ORC_A, temperature, deterministic,
                                action_u ? action_u[b] : 0.0, powtab, p);
      if (act < 0) status = -2;
      if (action) action[b] = act;
      if (pi) memcpy(pi + (size_t)b * ORC_A, p, sizeof(p));
    }
  }
  free(table); free(nodes); free(hbuf);
  return status;
}
