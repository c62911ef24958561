// mzh_rng.cpp -- host (CPU) restatement of the NumPy legacy RandomState draws one run_mcts call
// makes, so B calls' worth of reference-order draws cost C time instead of 3 NumPy calls per root.
//
// Reference consumption per run_mcts call, all on NumPy's global legacy
// MT19937 stream:
//   np.random.dirichlet(np.ones_like(prob) * alpha)    MCTS/mcts.py:57-66,148-149 (prob float32)
//   np.random.choice(np.where(ucb == max)[0])           MCTS/node.py:86 -- the root's first
//                                                       selection, always a 6-way tie
//   np.random.choice(np.arange(6), p=pi)                MCTS/mcts.py:118-120 (one random_sample)
// The algorithms restated are NumPy's published legacy ones (numpy 2.2 as installed here; the
// legacy RandomState stream is frozen across NumPy versions, the reason `legacy` exists):
//   - MT19937 (mt19937_gen / mt19937_next32 with tempering) and next_double = (a>>5, b>>6) / 2^53;
//   - RandomState.dirichlet: k legacy_standard_gamma(alpha_j) draws, acc summed in order,
//     invacc = 1/acc, each value * invacc;
//   - legacy_standard_gamma: shape == 1 -> legacy exponential -log(1 - U); shape < 1 ->
//     Johnk/Ahrens-Dieter rejection on (U, exponential V); shape > 1 -> Marsaglia-Tsang on the
//     legacy polar Gaussian (with its cached second deviate, the aug state's has_gauss / gauss);
//   - RandomState.choice(a) without p = randint(0, len(a)): masked rejection on 32-bit draws
//     (mask = next power of two - 1 above len - 1; draw & mask until <= len - 1);
//   - random_sample = next_double.
// The MT19937 state is NumPy's own (mt19937_state: uint32 key[624]; int pos), passed by address
// from the RandomState's bit generator (muzero-hanoi_amd/rng.py), so the stream advances in place.
// Compiled by g++ with -ffp-contract=off and without -march (no FMA), calling the same glibc
// log / pow / sqrt NumPy's C code calls; tests/test_rng_fast.py checks every array and the
// post-draw stream state against NumPy itself.
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/mzh.h"

namespace {

constexpr int kN = 624, kM = 397;

struct MtState {  // numpy/random/src/mt19937/mt19937.h: mt19937_state
  uint32_t key[kN];
  int pos;
};

void mt_gen(MtState* s) {
  const uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kA = 0x9908b0dfu;
  uint32_t y;
  int i = 0;
  for (; i < kN - kM; i++) {
    y = (s->key[i] & kUpper) | (s->key[i + 1] & kLower);
    s->key[i] = s->key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kA);
  }
  for (; i < kN - 1; i++) {
    y = (s->key[i] & kUpper) | (s->key[i + 1] & kLower);
    s->key[i] = s->key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kA);
  }
  y = (s->key[kN - 1] & kUpper) | (s->key[0] & kLower);
  s->key[kN - 1] = s->key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kA);
  s->pos = 0;
}

struct Stream {
  MtState* s;
  int has_gauss;
  double gauss;

  inline uint32_t next32() {
    if (s->pos == kN) mt_gen(s);
    uint32_t y = s->key[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  inline double next_double() {
    int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  inline double exponential() { return -log(1.0 - next_double()); }
  double polar_gauss() {
    if (has_gauss) {
      const double t = gauss;
      has_gauss = 0;
      gauss = 0.0;
      return t;
    }
    double f, x1, x2, r2;
    do {
      x1 = 2.0 * next_double() - 1.0;
      x2 = 2.0 * next_double() - 1.0;
      r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    f = sqrt(-2.0 * log(r2) / r2);
    gauss = f * x1;
    has_gauss = 1;
    return f * x2;
  }
  double standard_gamma(double shape) {
    if (shape == 1.0) return exponential();
    if (shape == 0.0) return 0.0;
    if (shape < 1.0) {
      for (;;) {
        const double U = next_double();
        const double V = exponential();
        if (U <= 1.0 - shape) {
          const double X = pow(U, 1. / shape);
          if (X <= V) return X;
        } else {
          const double Y = -log((1 - U) / shape);
          const double X = pow(1.0 - shape + shape * Y, 1. / shape);
          if (X <= (V + Y)) return X;
        }
      }
    }
    const double b = shape - 1. / 3.;
    const double c = 1. / sqrt(9 * b);
    for (;;) {
      double X, V;
      do {
        X = polar_gauss();
        V = 1.0 + c * X;
      } while (V <= 0.0);
      V = V * V * V;
      const double U = next_double();
      if (U < 1.0 - 0.0331 * (X * X) * (X * X)) return b * V;
      if (log(U) < 0.5 * X * X + b * (1. - V + log(V))) return b * V;
    }
  }
  // randint(0, n) with the legacy masked rejection (n - 1 <= 0xFFFFFFFE); n == 1 draws nothing
  inline int32_t bounded(uint32_t n) {
    const uint32_t rng = n - 1;
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > rng) {
    }
    return (int32_t)v;
  }
};

}  // namespace

/* include/mzh.h: mzh_rng_predraw */
extern "C" int mzh_rng_predraw(void* mt_state, double* gauss_state, int B, int k, const double* alpha,
                               int n_tie, int draw_action, double* noise, int32_t* tie, double* action_u) {
  if (!mt_state || !gauss_state || B < 0 || k < 0 || k > 64 || (k > 0 && (!alpha || !noise)) || n_tie < 0 ||
      (n_tie > 0 && !tie) || (draw_action && !action_u))
    return MZH_ERR_ARG;
  for (int j = 0; j < k; j++)
    if (!(alpha[j] > 0.0)) return MZH_ERR_ARG;  // RandomState.dirichlet: ValueError('alpha <= 0')
  Stream st{static_cast<MtState*>(mt_state), gauss_state[0] != 0.0 ? 1 : 0, gauss_state[1]};
  if (st.s->pos < 0 || st.s->pos > kN) return MZH_ERR_ARG;
  for (int r = 0; r < B; r++) {
    if (k > 0) {
      double* v = noise + (size_t)r * k;
      double acc = 0.;
      for (int j = 0; j < k; j++) {
        v[j] = st.standard_gamma(alpha[j]);
        acc = acc + v[j];
      }
      const double invacc = 1 / acc;
      for (int j = 0; j < k; j++) v[j] = v[j] * invacc;
    }
    if (n_tie > 0) tie[r] = st.bounded((uint32_t)n_tie);
    if (draw_action) action_u[r] = st.next_double();
  }
  gauss_state[0] = st.has_gauss ? 1.0 : 0.0;
  gauss_state[1] = st.gauss;
  return MZH_OK;
}
