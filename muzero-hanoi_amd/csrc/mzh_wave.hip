// mzh_wave.hip -- wave-independent fused batched search for large root batches (gfx950).
//
// Every wave owns 32 roots (two 16-root MFMA column tiles) and runs all of their simulations on
// its own: no __syncthreads after start-up, so the two waves a SIMD holds drift apart and one
// wave's latency-bound tree phase (select / backup: dependent L2 loads, fp64) overlaps the other
// wave's MFMA phase.  The MLPs run "transposed": the weights are the MFMA A operand (streamed
// from L2, one float4 per lane feeds 4 k-steps x 2 column tiles) and the activations are the B
// operand with one root per column, so a hidden tile's C registers are directly the next layer's
// B operand (MzhWMlp row permutation, mzh_internal.h) -- activations never touch LDS.
//
// Numerics are the contract of mzh_device.h unchanged: k-ordered fp32 FMA chains from 0 (bias
// after), mzh_expf softmax with the 8-partial summation order of oracle/mzh_oracle.c sum8_tree
// (the value/reward logits are permuted so that lane group g holds partials q = 2g, 2g+1), fp64
// tree statistics in MCTS/node.py's order.  Results are bit-identical to mzh_search_kernel.
//
// Reference: MCTS/mcts.py:34-126 (run_mcts), MCTS/node.py:30-136 (expand/backup/best_child),
// MCTS/utils_mcts.py:1-16 (MinMaxStats), networks.py:71-196 (initial/recurrent inference).
#include "mzh_device.h"
#include "mzh_internal.h"

#ifndef MZW_WAVES
#define MZW_WAVES 4   // waves per workgroup (independent after the start-up barrier)
#endif
#ifndef MZW_STAGGER
#define MZW_STAGGER 0  // start delay (s_sleep units of 64 cycles) of the second wave of each SIMD
#endif
#define MZW_NT 2      // 16-root column tiles per wave
#define MZW_ROOTS 32  // roots per wave
#define MZW_DC 16     // selection-path depths cached in LDS per root (deeper: HBM pathx)
#ifndef MZW_PIN
#define MZW_PIN 1     // pin the weight prefetch one hidden block ahead (sched_barrier)
#endif
#ifndef MZW_UNROLL
#define MZW_UNROLL 2
#endif
#define MZW_STR(x) #x
#define MZW_XSTR(x) MZW_STR(x)
#define MZW_UNROLL_PRAGMA _Pragma(MZW_XSTR(unroll MZW_UNROLL))
#ifndef MZW_FENCE
#define MZW_FENCE 1   // 1: workgroup-scope fence at the end of each simulation, 0: wavefront scope
#endif

// tree block: identical to mzh_search.hip's MzhBlock (one 128-B line per expanded node)
struct MzwNX {
  uint16_t N;
  int16_t X;
};
struct __align__(128) MzwBlock {
  MzwNX nx[6];
  float R[6];
  float P[6];
  double W[6];
  uint32_t pad[2];
};
static_assert(sizeof(MzwBlock) == 128, "block layout");

// per-wave LDS: the roots' own children (SoA, lane = root: conflict-free) and the path cache
struct MzwWave {
  double rW[6][MZW_ROOTS];
  double rP[6][MZW_ROOTS];  // fp64 prior (Dirichlet-mixed or the widened fp32 prior)
  float rR[6][MZW_ROOTS];
  int rN[6][MZW_ROOTS];
  int rX[6][MZW_ROOTS];
  double pcW[MZW_DC][MZW_ROOTS];  // chosen child's statistics at each depth (select snapshot)
  float pcR[MZW_DC][MZW_ROOTS];
  int pcN[MZW_DC][MZW_ROOTS];
  uint16_t path[MZW_DC][MZW_ROOTS];  // slot = parent expanded index * 8 + child
};

static __host__ __device__ inline size_t mzw_hdr_bytes(int S) {
  size_t b = sizeof(float) * MZH_A * MZH_F + sizeof(double) * 2 * (size_t)(S + 3);
  return (b + 15) & ~(size_t)15;
}

__device__ __forceinline__ void mzw_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float mzw_max4g(float v) {  // max over the 4 lane groups of a column
  float t = __shfl_xor(v, 16);
  v = t > v ? t : v;
  t = __shfl_xor(v, 32);
  return t > v ? t : v;
}
__device__ __forceinline__ float mzw_min4g(float v) {
  float t = __shfl_xor(v, 16);
  v = t < v ? t : v;
  t = __shfl_xor(v, 32);
  return t < v ? t : v;
}

// ------------------------------------------------------------------------------------------
// One MLP (layer1 + bias (+ one-hot column) + ReLU -> layer2, bias2 left to the caller) for the
// wave's 2 column tiles.  x[n][kb] = the B operand of column tile n, k-block kb (lane group g
// holds inputs 16kb + 4t + g, t = 0..3).  out[ot][n]: C registers of output tile ot.
// ------------------------------------------------------------------------------------------
template <int KB1, int NO, bool OH>
__device__ __forceinline__ void mzw_chain(const MzhWMlp& L, const floatx4 (&x)[MZW_NT][4], const float* oh0,
                                          const float* oh1, floatx4 (&out)[NO][MZW_NT], int lane) {
  constexpr int FR = KB1 + NO;
  const int g = lane >> 4;
  const floatx4* S = reinterpret_cast<const floatx4*>(L.s) + lane;
  const float* B1 = L.b1 + 4 * g;
#pragma unroll
  for (int ot = 0; ot < NO; ++ot)
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n) out[ot][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 w[FR], b, o[MZW_NT];
#pragma unroll
  for (int f = 0; f < FR; ++f) w[f] = S[f * 64];
  b = *reinterpret_cast<const floatx4*>(B1);
#pragma unroll
  for (int n = 0; n < MZW_NT; ++n)
    o[n] = OH ? *reinterpret_cast<const floatx4*>(n == 0 ? oh0 : oh1) : floatx4{0.f, 0.f, 0.f, 0.f};
  MZW_UNROLL_PRAGMA
  for (int ht = 0; ht < 16; ++ht) {
    // next block's fragments, bias and one-hot columns: issued here and kept in flight across
    // this block's MFMAs (the scheduling barrier stops the compiler from sinking the loads to
    // their uses, which would expose the L2 latency once per fragment)
    floatx4 wn[FR], bn, on[MZW_NT];
#pragma unroll
    for (int f = 0; f < FR; ++f) wn[f] = S[((ht + 1) * FR + f) * 64];  // block 16 is the zero pad
    bn = *reinterpret_cast<const floatx4*>(B1 + 16 * ((ht + 1) & 15));
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n)
      on[n] = OH ? *reinterpret_cast<const floatx4*>((n == 0 ? oh0 : oh1) + 16 * ((ht + 1) & 15))
                 : floatx4{0.f, 0.f, 0.f, 0.f};
    if (MZW_PIN) __builtin_amdgcn_sched_barrier(0);
    floatx4 acc[MZW_NT];
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n) acc[n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB1; ++kb)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int n = 0; n < MZW_NT; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[kb][t], x[n][kb][t], acc[n], 0, 0, 0);
    floatx4 hid[MZW_NT];
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[n][i];
        if (OH) v = v + o[n][i];  // one-hot action column (k = 64 + a)
        v = v + b[i];
        hid[n][i] = v > 0.0f ? v : 0.0f;
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int ot = 0; ot < NO; ++ot)
#pragma unroll
        for (int n = 0; n < MZW_NT; ++n)
          out[ot][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[KB1 + ot][t], hid[n][t], out[ot][n], 0, 0, 0);
#pragma unroll
    for (int f = 0; f < FR; ++f) w[f] = wn[f];
    b = bn;
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n) o[n] = on[n];
  }
}

template <int NO>
__device__ __forceinline__ void mzw_bias2(const MzhWMlp& L, floatx4 (&out)[NO][MZW_NT], int g) {
#pragma unroll
  for (int ot = 0; ot < NO; ++ot) {
    const floatx4 b = *reinterpret_cast<const floatx4*>(L.b2 + 16 * ot + 4 * g);
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) out[ot][n][i] = out[ot][n][i] + b[i];
  }
}

// normalize_h_state (networks.py:191-196) of one column: lane group g holds 16 of the 64 units
__device__ __forceinline__ void mzw_normalize(const floatx4 (&hp)[4][MZW_NT], int n, floatx4 (&hn)[MZW_NT][4]) {
  float mn = hp[0][n][0], mx = hp[0][n][0];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = hp[ot][n][i];
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
    }
  mn = mzw_min4g(mn);
  mx = mzw_max4g(mx);
  const float d = (mx - mn) + 9.999999939225290290778502821922302246094e-09f;
  const float y = 1.0f / d;
  bool slow = false;
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) hn[n][ot][i] = mzh_fdiv(hp[ot][n][i] - mn, d, y, slow);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
#pragma unroll
    for (int ot = 0; ot < 4; ++ot)
#pragma unroll
      for (int i = 0; i < 4; ++i) hn[n][ot][i] = (hp[ot][n][i] - mn) / d;
  }
}

// logits_to_transformed_expected_value (networks.py:152-189) for one column of a 33-bin head.
// Slot s = 4ot + i of lane group g holds logit k = 2g + (s & 1) + 8(s >> 1) (slot 8 only for g = 0),
// so the lane's two sequential partials are the oracle's s_{2g}, s_{2g+1} and the cross-group
// adds reproduce ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)).
template <int NO>
__device__ __forceinline__ float mzw_head(const floatx4 (&l)[NO][MZW_NT], int n, int lane) {
  const int g = lane >> 4;
  if constexpr (NO == 1) {
    return __shfl(l[0][n][0], lane & 15);  // support 1: the raw logit (networks.py:146-148)
  } else {
  const bool v8 = g == 0;
  float L[9];
#pragma unroll
  for (int s = 0; s < 9; ++s) L[s] = l[s >> 2][n][s & 3];
  float m = L[0];
#pragma unroll
  for (int s = 1; s < 8; ++s) m = L[s] > m ? L[s] : m;
  if (v8) m = L[8] > m ? L[8] : m;
  m = mzw_max4g(m);
  float e[9];
#pragma unroll
  for (int s = 0; s < 8; ++s) e[s] = mzh_expf(L[s] - m);
  e[8] = v8 ? mzh_expf(L[8] - m) : 0.0f;
  float s0 = e[0];
  s0 = s0 + e[2];
  s0 = s0 + e[4];
  s0 = s0 + e[6];
  if (v8) s0 = s0 + e[8];
  float s1 = e[1];
  s1 = s1 + e[3];
  s1 = s1 + e[5];
  s1 = s1 + e[7];
  float t = s0 + s1;
  t = t + __shfl_xor(t, 16);
  t = t + __shfl_xor(t, 32);
  const float y = 1.0f / t;
  bool slow = false;
  float pk[9];
#pragma unroll
  for (int s = 0; s < 9; ++s) pk[s] = mzh_fdiv(e[s], t, y, slow);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
#pragma unroll
    for (int s = 0; s < 9; ++s) pk[s] = e[s] / t;
  }
  float pr[9];
#pragma unroll
  for (int s = 0; s < 9; ++s) pr[s] = pk[s] * (float)(2 * g + (s & 1) + 8 * (s >> 1) - 16);
  float x0 = pr[0];
  x0 = x0 + pr[2];
  x0 = x0 + pr[4];
  x0 = x0 + pr[6];
  if (v8) x0 = x0 + pr[8];
  float x1 = pr[1];
  x1 = x1 + pr[3];
  x1 = x1 + pr[5];
  x1 = x1 + pr[7];
  float xs = x0 + x1;
  xs = xs + __shfl_xor(xs, 16);
  xs = xs + __shfl_xor(xs, 32);
  return mzh_signed_parabolic(xs);
  }
}

// softmax of the 6 policy logits (networks.py:83,109): lane group 0 holds logits 0-3, group 1
// logits 4-5 (registers 0,1); returns the probabilities in the same registers
__device__ __forceinline__ floatx4 mzw_policy(const floatx4 l, int lane) {
  const int g = lane >> 4;
  const bool ok01 = g < 2, ok23 = g == 0;
  float m = -__builtin_inff();
  if (ok01) {
    m = l[0] > m ? l[0] : m;
    m = l[1] > m ? l[1] : m;
  }
  if (ok23) {
    m = l[2] > m ? l[2] : m;
    m = l[3] > m ? l[3] : m;
  }
  m = mzw_max4g(m);
  const float e0 = ok01 ? mzh_expf(l[0] - m) : 0.0f, e1 = ok01 ? mzh_expf(l[1] - m) : 0.0f;
  const float e2 = ok23 ? mzh_expf(l[2] - m) : 0.0f, e3 = ok23 ? mzh_expf(l[3] - m) : 0.0f;
  float t = (e0 + e1) + (e2 + e3);
  t = t + __shfl_xor(t, 16);  // group 0: ((s0+s1)+(s2+s3)) + ((s4+s5)+(0+0))
  const float y = 1.0f / t;
  bool slow = false;
  floatx4 p;
  p[0] = mzh_fdiv(e0, t, y, slow);
  p[1] = mzh_fdiv(e1, t, y, slow);
  p[2] = mzh_fdiv(e2, t, y, slow);
  p[3] = mzh_fdiv(e3, t, y, slow);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    p[0] = e0 / t;
    p[1] = e1 / t;
    p[2] = e2 / t;
    p[3] = e3 / t;
  }
  return p;
}

// ---- tree helpers (same arithmetic as mzh_search.hip) ----
__device__ __forceinline__ double mzw_div(double a, double b, double y) {
  const double q = a * y;
  const double r = __builtin_fma(-q, b, a);
  return __builtin_fma(r, y, q);
}
__device__ __forceinline__ float mzw_ucb(int Nc, double Wc, float Rc, double P64, bool p64_semantics, double tnp,
                                         double disc, bool has, double mn, double den, double dinv,
                                         const double* inv) {
  float q32 = 0.0f;
  if (Nc > 0) {
    const double v = (double)Rc + disc * mzw_div(Wc, (double)Nc, inv[Nc]);
    q32 = (float)(has ? mzw_div(v - mn, den, dinv) : v);
  }
  const double w = mzw_div(tnp, (double)(Nc + 1), inv[Nc + 1]);
  const float u32 = p64_semantics ? (float)(P64 * w) : (float)P64 * (float)w;
  return q32 + u32;
}
// in-lane argmax over 6 children with the reference's tie handling (see mzh_group_pick)
__device__ __forceinline__ int mzw_pick(const float (&u)[6], int tie, int& firstTie, int& extra) {
  float m = u[0];
#pragma unroll
  for (int c = 1; c < 6; ++c) m = u[c] > m ? u[c] : m;
  int mask = 0;
#pragma unroll
  for (int c = 0; c < 6; ++c) mask |= (u[c] == m ? 1 : 0) << c;
  const int cnt = __popc(mask);
  const int first = __ffs(mask) - 1;
  const bool six = (cnt == MZH_A) & (firstTie == 0);
  extra += ((cnt > 1) & !six) ? 1 : 0;
  firstTie |= six ? 1 : 0;
  return six ? tie : first;
}

template <bool REPLAY, bool SUP33>
__global__ __launch_bounds__(MZW_WAVES * 64, 8 / MZW_WAVES) void mzh_wave_kernel(MzhWNet net, MzhSearchParams p) {
  constexpr int NOV = SUP33 ? 3 : 1;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int S = p.S;
  float* ohl = reinterpret_cast<float*>(smem_raw);
  double* table = reinterpret_cast<double*>(smem_raw + sizeof(float) * MZH_A * MZH_F);
  double* inv = table + (S + 3);
  MzwWave* wsa = reinterpret_cast<MzwWave*>(smem_raw + mzw_hdr_bytes(S));
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, col = lane & 15;

  if (!REPLAY)
    for (int i = tid; i < MZH_A * MZH_F; i += MZW_WAVES * 64) ohl[i] = net.oh[i];
  for (int i = tid; i < S + 3; i += MZW_WAVES * 64) {
    table[i] = i < S + 2 ? p.table[i] : 0.0;
    inv[i] = 1.0 / (double)i;  // IEEE division: correctly rounded
  }
  __syncthreads();  // the only barrier: from here on every wave runs independently
  if (MZW_STAGGER > 0 && wave >= 4) {
    // waves w and w + 4 share a SIMD: start the second one about a tree phase later so the two
    // alternate between MFMA and tree work instead of running their phases in lockstep
    for (int i = 0; i < MZW_STAGGER / 127; ++i) __builtin_amdgcn_s_sleep(127);
  }
  const int wr0 = (blockIdx.x * MZW_WAVES + wave) * MZW_ROOTS;
  if (wr0 >= p.B) return;
  MzwWave& ws = wsa[wave];
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;
  const size_t E = (size_t)p.E;

  // root lanes: lane rho < 32 owns root wr0 + rho (tree phases)
  const int rho = lane;
  const int rroot = wr0 + rho;
  const bool rvalid = lane < MZW_ROOTS && rroot < p.B;
  MzwBlock* tb = reinterpret_cast<MzwBlock*>(p.tree) + (size_t)(rvalid ? rroot : 0) * E;
  double mmax = -__builtin_inf(), mmin = __builtin_inf();
  if (rvalid && p.minmax_in) {
    mmax = p.minmax_in[2 * rroot];
    mmin = p.minmax_in[2 * rroot + 1];
  }
  double den = mmax - mmin, dinv = mmax > mmin ? 1.0 / (mmax - mmin) : 0.0;
  int firstTie = 0, extra = 0, steps = 0, rootN = 0, depth = 0, leafE = 0, leafA = 0;
  double rootW = 0.0;
  const int tie = (rvalid && p.tie_idx) ? p.tie_idx[rroot] : 0;

  // column lanes: lane (g, col) works on root wr0 + 16n + col of column tile n (MLP phases)
  int croot[MZW_NT];
  bool cvalid[MZW_NT];
#pragma unroll
  for (int n = 0; n < MZW_NT; ++n) {
    croot[n] = wr0 + 16 * n + col;
    cvalid[n] = croot[n] < p.B;
  }

  floatx4 hreg[MZW_NT][4];  // normalised latent of the newest expanded node (B-operand order)
#pragma unroll
  for (int n = 0; n < MZW_NT; ++n)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) hreg[n][kb] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---------------- root: initial_inference (mcts.py:49-50) + root.expand (mcts.py:57-69) ----------------
  floatx4 rpi[MZW_NT];
  if (!REPLAY) {
    floatx4 x[MZW_NT][4];
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = 16 * kb + 4 * t + g;
          x[n][kb][t] = (cvalid[n] && k < p.in_dim) ? p.obs[(size_t)croot[n] * p.in_dim + k] : 0.0f;
        }
    floatx4 hp[4][MZW_NT];
    switch (net.rep.kb1) {
      case 1: mzw_chain<1, 4, false>(net.rep, x, nullptr, nullptr, hp, lane); break;
      case 2: mzw_chain<2, 4, false>(net.rep, x, nullptr, nullptr, hp, lane); break;
      case 3: mzw_chain<3, 4, false>(net.rep, x, nullptr, nullptr, hp, lane); break;
      default: mzw_chain<4, 4, false>(net.rep, x, nullptr, nullptr, hp, lane); break;
    }
    mzw_bias2<4>(net.rep, hp, g);
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n) {
      mzw_normalize(hp, n, hreg);
      if (cvalid[n]) {
        floatx4* dst = reinterpret_cast<floatx4*>(p.htree + ((size_t)croot[n] * E) * MZH_H) + g;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) dst[4 * kb] = hreg[n][kb];
      }
    }
    floatx4 pl[1][MZW_NT];
    mzw_chain<4, 1, false>(net.pol, hreg, nullptr, nullptr, pl, lane);
    mzw_bias2<1>(net.pol, pl, g);
    floatx4 vl[NOV][MZW_NT];
    mzw_chain<4, NOV, false>(net.val, hreg, nullptr, nullptr, vl, lane);  // root value: computed, unused (mcts.py:50)
    (void)vl;
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n) rpi[n] = mzw_policy(pl[0][n], lane);
  }
  // root children: prior (Dirichlet-mixed when noised), N = 0, unexpanded
  if (g < 2) {
#pragma unroll
    for (int n = 0; n < MZW_NT; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * g + i;
        if (c < MZH_A && cvalid[n]) {
          const float pr = REPLAY ? p.rp_root_pi[(size_t)croot[n] * MZH_A + c] : rpi[n][i];
          double v = (double)pr;
          if (noised) {
            const float scaled = (float)(1.0 - p.eps) * pr;  // (1-eps) * prob, float32 array
            v = (double)scaled + p.eps * p.noise[(size_t)croot[n] * MZH_A + c];
          }
          ws.rP[c][16 * n + col] = v;
        }
      }
  }
  if (lane < MZW_ROOTS) {
#pragma unroll
    for (int c = 0; c < MZH_A; ++c) {
      ws.rW[c][rho] = 0.0;
      ws.rR[c][rho] = 0.0f;
      ws.rN[c][rho] = 0;
      ws.rX[c][rho] = -1;
    }
  }
  mzw_wave_sync();

  MZH_STAMP_DECL
  for (int s = 0; s < S; ++s) {
    MZH_STAMP(0);
    // ---------------- select (mcts.py:75-86; node.py:72-123): one lane per root ----------------
    if (rvalid) {
      const bool has = mmax > mmin;
      float u[6];
      const double tr = table[rootN];
#pragma unroll
      for (int c = 0; c < MZH_A; ++c)
        u[c] = mzw_ucb(ws.rN[c][rho], ws.rW[c][rho], ws.rR[c][rho], ws.rP[c][rho], noised || p.np1, tr, disc, has,
                       mmin, den, dinv, inv);
      int pick = mzw_pick(u, tie, firstTie, extra);
      int Np = ws.rN[pick][rho], X = ws.rX[pick][rho];
      ws.path[0][rho] = (uint16_t)pick;
      ws.pcW[0][rho] = ws.rW[pick][rho];
      ws.pcR[0][rho] = ws.rR[pick][rho];
      ws.pcN[0][rho] = Np;
      int e = 0, d = 1;
      while (X >= 0 && d <= S) {  // depth <= s + 1 always; the bound only guards against a corrupt tree
        e = X;
        const int4* bp = reinterpret_cast<const int4*>(tb + e);
        int dw[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int4 q = bp[k];
          dw[4 * k] = q.x;
          dw[4 * k + 1] = q.y;
          dw[4 * k + 2] = q.z;
          dw[4 * k + 3] = q.w;
        }
        double Wc[6];
        float Rc[6];
#pragma unroll
        for (int c = 0; c < MZH_A; ++c) {
          Rc[c] = __int_as_float(dw[6 + c]);
          Wc[c] = __hiloint2double(dw[19 + 2 * c], dw[18 + 2 * c]);
          u[c] = mzw_ucb(dw[c] & 0xFFFF, Wc[c], Rc[c], (double)__int_as_float(dw[12 + c]), p.np1, table[Np], disc,
                         has, mmin, den, dinv, inv);
        }
        pick = mzw_pick(u, tie, firstTie, extra);
        int nx = dw[0];
        double Wp = Wc[0];
        float Rp = Rc[0];
#pragma unroll
        for (int c = 1; c < MZH_A; ++c)
          if (pick == c) {
            nx = dw[c];
            Wp = Wc[c];
            Rp = Rc[c];
          }
        Np = nx & 0xFFFF;
        X = nx >> 16;
        const uint16_t slot = (uint16_t)(e * 8 + pick);
        if (d < MZW_DC) {
          ws.path[d][rho] = slot;
          ws.pcW[d][rho] = Wp;
          ws.pcR[d][rho] = Rp;
          ws.pcN[d][rho] = Np;
        } else {
          p.pathx[(size_t)rroot * E + d] = slot;
        }
        ++d;
      }
      depth = d;
      leafE = e;
      leafA = pick;
      steps += d;
    }
    MZH_STAMP(1);

    // ---------------- expand via the network (mcts.py:88-106) ----------------
    float val[MZW_NT], rew[MZW_NT];
    floatx4 cpi[MZW_NT];
    if (!REPLAY) {
      int en[MZW_NT], an[MZW_NT];
#pragma unroll
      for (int n = 0; n < MZW_NT; ++n) {
        en[n] = __shfl(leafE, 16 * n + col);
        an[n] = __shfl(leafA, 16 * n + col);
      }
      // parent latent (mcts.py:89-92): the node expanded by the previous simulation is in hreg
      floatx4 x[MZW_NT][4];
#pragma unroll
      for (int n = 0; n < MZW_NT; ++n) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) x[n][kb] = hreg[n][kb];
        if (cvalid[n] && en[n] != s) {
          const floatx4* src = reinterpret_cast<const floatx4*>(p.htree + ((size_t)croot[n] * E + en[n]) * MZH_H) + g;
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) x[n][kb] = src[4 * kb];
        }
      }
      MZH_STAMP(2);
      floatx4 hp[4][MZW_NT];
      mzw_chain<4, 4, true>(net.dyn, x, ohl + an[0] * MZH_F + 4 * g, ohl + an[1] * MZH_F + 4 * g, hp, lane);
      mzw_bias2<4>(net.dyn, hp, g);  // h' (un-normalised, networks.py:129-138)
      MZH_STAMP(3);
      floatx4 hx[MZW_NT][4];
#pragma unroll
      for (int n = 0; n < MZW_NT; ++n)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) hx[n][kb] = hp[kb][n];
      {
        floatx4 rl[NOV][MZW_NT];
        mzw_chain<4, NOV, false>(net.rwd, hx, nullptr, nullptr, rl, lane);  // reward from h' (networks.py:132-135)
        mzw_bias2<NOV>(net.rwd, rl, g);
        MZH_STAMP(4);
#pragma unroll
        for (int n = 0; n < MZW_NT; ++n) rew[n] = mzw_head<NOV>(rl, n, lane);
      }
      MZH_STAMP(5);
#pragma unroll
      for (int n = 0; n < MZW_NT; ++n) {
        mzw_normalize(hp, n, hreg);
        if (cvalid[n]) {
          floatx4* dst = reinterpret_cast<floatx4*>(p.htree + ((size_t)croot[n] * E + s + 1) * MZH_H) + g;
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) dst[4 * kb] = hreg[n][kb];
        }
      }
      MZH_STAMP(6);
      {
        floatx4 pl[1][MZW_NT];
        mzw_chain<4, 1, false>(net.pol, hreg, nullptr, nullptr, pl, lane);
        mzw_bias2<1>(net.pol, pl, g);
        MZH_STAMP(7);
#pragma unroll
        for (int n = 0; n < MZW_NT; ++n) cpi[n] = mzw_policy(pl[0][n], lane);
      }
      MZH_STAMP(8);
      {
        floatx4 vl[NOV][MZW_NT];
        mzw_chain<4, NOV, false>(net.val, hreg, nullptr, nullptr, vl, lane);
        mzw_bias2<NOV>(net.val, vl, g);
        MZH_STAMP(9);
#pragma unroll
        for (int n = 0; n < MZW_NT; ++n) val[n] = mzw_head<NOV>(vl, n, lane);
      }
      MZH_STAMP(10);
      // the new node's 6 children (node.py:44-49): lane groups 0/1 hold pi[0..3] / pi[4..5]
      if (g < 2) {
#pragma unroll
        for (int n = 0; n < MZW_NT; ++n) {
          if (!cvalid[n]) continue;
          MzwBlock* nb = reinterpret_cast<MzwBlock*>(p.tree) + (size_t)croot[n] * E + (s + 1);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = 4 * g + i;
            if (c < MZH_A) {
              *reinterpret_cast<uint32_t*>(&nb->nx[c]) = 0xFFFF0000u;  // N = 0, X = -1
              nb->R[c] = 0.0f;
              nb->P[c] = cpi[n][i];
              nb->W[c] = 0.0;
            }
          }
        }
      }
    }

    MZH_STAMP(11);
    // ---------------- expand bookkeeping + backup (node.py:30-70): one lane per root ----------------
    if (rvalid) {
      const int enew = s + 1;
      float vv, rr;
      if (REPLAY) {
        vv = p.rp_value[(size_t)rroot * S + s];
        rr = p.rp_reward[(size_t)rroot * S + s];
        MzwBlock* nb = tb + enew;
#pragma unroll
        for (int c = 0; c < MZH_A; ++c) {
          *reinterpret_cast<uint32_t*>(&nb->nx[c]) = 0xFFFF0000u;
          nb->R[c] = 0.0f;
          nb->P[c] = p.rp_pi[((size_t)rroot * S + s) * MZH_A + c];
          nb->W[c] = 0.0;
        }
      } else {
        vv = lane < 16 ? val[0] : val[1];  // lane rho < 16: tile 0 column rho; 16..31: tile 1
        rr = lane < 16 ? rew[0] : rew[1];
      }
      if (leafE == 0) {
        ws.rX[leafA][rho] = enew;
        ws.rR[leafA][rho] = rr;
      } else {
        tb[leafE].nx[leafA].X = (int16_t)enew;
        tb[leafE].R[leafA] = rr;
      }
      double v = (double)vv;
      double lmax = -__builtin_inf(), lmin = __builtin_inf();
      for (int j = depth - 1; j >= 0; --j) {
        const int slot = j < MZW_DC ? (int)ws.path[j][rho] : (int)p.pathx[(size_t)rroot * E + j];
        const int e = slot >> 3, a = slot & 7;
        double Wj;
        float Rj;
        int Nj;
        if (j < MZW_DC) {
          Wj = ws.pcW[j][rho];
          Rj = ws.pcR[j][rho];
          Nj = ws.pcN[j][rho];
        } else {
          Wj = tb[e].W[a];
          Rj = tb[e].R[a];
          Nj = tb[e].nx[a].N;
        }
        const double rw = (j == depth - 1) ? (double)rr : (double)Rj;
        const double Wn = Wj + v;
        const int Nn = Nj + 1;
        if (e == 0) {
          ws.rW[a][rho] = Wn;
          ws.rN[a][rho] = Nn;
        } else {
          tb[e].W[a] = Wn;
          tb[e].nx[a].N = (uint16_t)Nn;
        }
        const double q = rw + disc * mzw_div(Wn, (double)Nn, inv[Nn]);
        lmax = q > lmax ? q : lmax;
        lmin = q < lmin ? q : lmin;
        v = rw + disc * v;
      }
      rootW = rootW + v;
      rootN = rootN + 1;
      const double q = 0.0 + disc * mzw_div(rootW, (double)rootN, inv[rootN]);  // root rwd = 0.0
      lmax = q > lmax ? q : lmax;
      lmin = q < lmin ? q : lmin;
      mmax = lmax > mmax ? lmax : mmax;
      mmin = lmin < mmin ? lmin : mmin;
      den = mmax - mmin;
      dinv = mmax > mmin ? 1.0 / (mmax - mmin) : 0.0;
    }
    MZH_STAMP(12);
    // this simulation's tree stores (other lanes' new-block writes) before the next selection
    if (MZW_FENCE)
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    else
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    MZH_STAMP(13);
  }

  // ---------------- results (mcts.py:111-126, 154-176) ----------------
  if (!rvalid) return;
  const int root = rroot;
  int vis[MZH_A];
  for (int a = 0; a < MZH_A; ++a) {
    vis[a] = ws.rN[a][rho];
    p.visits[(size_t)root * MZH_A + a] = vis[a];
  }
  if (p.root_q) p.root_q[root] = rootN == 0 ? 0.0 : rootW / (double)rootN;
  if (p.minmax_out) {
    p.minmax_out[2 * root] = mmax;
    p.minmax_out[2 * root + 1] = mmin;
  }
  if (p.extra_ties) p.extra_ties[root] = extra;
  if (p.sel_steps) p.sel_steps[root] = steps;
  const int PL = S + 1;
  if (p.latent && S > 0) {
    for (int j = 0; j < depth; ++j)
      p.latent[(size_t)root * PL + j] = (j < MZW_DC ? (int)ws.path[j][rho] : (int)p.pathx[(size_t)root * E + j]) & 7;
    for (int j = depth; j < PL; ++j) p.latent[(size_t)root * PL + j] = -1;
  }
  if (p.latent_len) p.latent_len[root] = S > 0 ? depth : 0;
  if (p.pi || p.action) {
    double v[MZH_A];
    for (int a = 0; a < MZH_A; ++a) v[a] = (double)vis[a];
    if (p.temperature > 0.0) {
      double ex = 1.0 / p.temperature;
      ex = ex < 5.0 ? ex : 5.0;  // max(1.0, min(5.0, 1/T))
      ex = ex > 1.0 ? ex : 1.0;
      for (int a = 0; a < MZH_A; ++a) {
        if (ex == __builtin_rint(ex)) {
          double r = v[a];
          for (int i = 1; i < (int)ex; ++i) r = r * v[a];
          v[a] = r;
        } else {
          v[a] = pow(v[a], ex);
        }
      }
    }
    double sum = 0.0;
    for (int a = 0; a < MZH_A; ++a) sum = sum + v[a];
    double pi[MZH_A];
    for (int a = 0; a < MZH_A; ++a) pi[a] = v[a] / sum;
    if (p.pi)
      for (int a = 0; a < MZH_A; ++a) p.pi[(size_t)root * MZH_A + a] = pi[a];
    int act = 0;
    if (p.deterministic || !p.action_u) {
      for (int a = 1; a < MZH_A; ++a)
        if (vis[a] > vis[act]) act = a;
    } else {
      double cdf[MZH_A];
      double acc = 0.0;
      for (int a = 0; a < MZH_A; ++a) {
        acc = acc + pi[a];
        cdf[a] = acc;
      }
      const double last = cdf[MZH_A - 1];
      const double u = p.action_u[root];
      act = MZH_A - 1;
      for (int a = 0; a < MZH_A; ++a) {
        if (cdf[a] / last > u) {
          act = a;
          break;
        }
      }
    }
    if (p.action) p.action[root] = act;
  }
}

size_t mzh_wave_smem_bytes(int S) { return mzw_hdr_bytes(S) + sizeof(MzwWave) * MZW_WAVES; }

template <bool REPLAY, bool SUP33>
static hipError_t launch_wave_t(const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const size_t smem = mzh_wave_smem_bytes(p.S);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mzh_wave_kernel<REPLAY, SUP33>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int per_wg = MZW_WAVES * MZW_ROOTS;
  const int grid = (p.B + per_wg - 1) / per_wg;
  hipLaunchKernelGGL((mzh_wave_kernel<REPLAY, SUP33>), dim3(grid), dim3(MZW_WAVES * 64), smem, stream, net, p);
  return hipGetLastError();
}

hipError_t mzh_launch_wave_search(bool replay, const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const bool sup33 = net.support == 33;
  if (replay) return sup33 ? launch_wave_t<true, true>(net, p, stream) : launch_wave_t<true, false>(net, p, stream);
  return sup33 ? launch_wave_t<false, true>(net, p, stream) : launch_wave_t<false, false>(net, p, stream);
}

#ifdef MZH_STAMPS
// diagnostic build only: this translation unit's phase stamps [8 waves][MZH_NSTAMP], read and cleared
extern "C" int mzh_diag_wave_stamps(unsigned long long* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(mzh_stamp_acc), sizeof(mzh_stamp_acc)) != hipSuccess) return -2;
  static unsigned long long zero[8][MZH_NSTAMP] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(mzh_stamp_acc), zero, sizeof(zero)) != hipSuccess) return -2;
  return 0;
}
#endif
