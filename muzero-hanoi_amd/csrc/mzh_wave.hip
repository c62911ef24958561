// mzh_wave.hip -- wave-independent fused batched search for large root batches (gfx950).
//
// Every wave owns 16*NT roots (NT 16-root MFMA column tiles) and runs all of their simulations on
// its own: no __syncthreads after start-up, so the two waves a SIMD holds drift apart and one
// wave's latency-bound tree phase (select / backup: dependent L2 loads, fp64) overlaps the other
// wave's MFMA phase.  The MLPs run "transposed": the weights are the MFMA A operand (streamed
// from L2, one float4 per lane feeds 4 k-steps x NT column tiles) and the activations are the B
// operand with one root per column, so a hidden tile's C registers are directly the next layer's
// B operand (MzhWMlp row permutation, mzh_internal.h) -- activations never touch LDS.
//
// Numerics are the contract of mzh_device.h unchanged: k-ordered fp32 FMA chains from 0 (bias
// after), mzh_expf softmax with the 8-partial summation order of oracle/mzh_oracle.c sum8_tree
// (the value/reward logits are permuted so that lane group g holds partials q = 2g, 2g+1), fp64
// tree statistics in MCTS/node.py's order.  Results are bit-identical to mzh_search_kernel.
//
// Schedule variants measured and not shipped (numbers in DESIGN.md §6/§8): an explicit ping-pong of
// the two waves per SIMD, software-pipelined MLP chains, LDS parking of the tree statistics,
// laundered weight pointers, cached child values in the tree block, a register reciprocal.  The
// child-block prefetch in selection is shipped for 16-root waves only (neutral at 32 roots per wave).
//
// Reference: MCTS/mcts.py:34-126 (run_mcts), MCTS/node.py:30-136 (expand/backup/best_child),
// MCTS/utils_mcts.py:1-16 (MinMaxStats), networks.py:71-196 (initial/recurrent inference).
#include "mzh_device.h"
#include "mzh_internal.h"

#define MZW_WAVES 4   // waves per workgroup; two workgroups per CU = two waves per SIMD (256 VGPRs)
#define MZW_DC 16     // selection-path depths cached in LDS per root (deeper: HBM pathx)

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
template <int ROOTS>
struct MzwWave {
  double rW[6][ROOTS];
  double rP[6][ROOTS];  // fp64 prior (Dirichlet-mixed or the widened fp32 prior)
  float rR[6][ROOTS];
  int rN[6][ROOTS];
  int rX[6][ROOTS];
  double pcW[MZW_DC][ROOTS];  // chosen child's statistics at each depth (select snapshot)
  float pcR[MZW_DC][ROOTS];
  int pcN[MZW_DC][ROOTS];
  uint16_t path[MZW_DC][ROOTS];  // slot = parent expanded index * 8 + child
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

// Cross-row exchange without LDS: v_permlane16_swap / v_permlane32_swap of a register with itself
// leave {own, partner} (rows r, r^1 resp. halves h, h^1) in the two results, in the same order on
// both lanes of a pair, so op(r[0], r[1]) is bit-identical on both (and equal to op(own, partner)
// for the commutative max / min / add used here).
__device__ __forceinline__ void mzw_pair16(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void mzw_pair32(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
// The maxima below feed only exponent arguments (x - max: identical for a +0 / -0 max), the
// normaliser's max - min (likewise) and argmax equality masks, and no operand is NaN: v_max_f32
// (one instruction) instead of compare + select (two, with a VCC hazard wait between them).
__device__ __forceinline__ float mzw_max4g(float v) {  // max over the 4 lane groups (rows) of a column
  float a, b;
  mzw_pair16(v, a, b);
  v = __builtin_fmaxf(a, b);
  mzw_pair32(v, a, b);
  return __builtin_fmaxf(a, b);
}
// min over the 4 lane groups for the latent normalisation: no operand is NaN or -0 (a latent unit is
// an FMA chain from +0 plus a bias, which never rounds to -0), so v_min_f32 is the select's result
__device__ __forceinline__ float mzw_min4g(float v) {
  float a, b;
  mzw_pair16(v, a, b);
  v = __builtin_fminf(a, b);
  mzw_pair32(v, a, b);
  return __builtin_fminf(a, b);
}
__device__ __forceinline__ float mzw_add16(float v) {  // row0 + row1 (row2 + row3)
  float a, b;
  mzw_pair16(v, a, b);
  return a + b;
}
__device__ __forceinline__ float mzw_add32(float v) {  // rows 0-1 + rows 2-3
  float a, b;
  mzw_pair32(v, a, b);
  return a + b;
}

// ------------------------------------------------------------------------------------------
// One MLP (layer1 + bias (+ one-hot column) + ReLU -> layer2, bias2 left to the caller) for the
// wave's NT column tiles.  x[n][kb] = the B operand of column tile n, k-block kb (lane group g
// holds inputs 16kb + 4t + g, t = 0..3).  out[ot][n]: C registers of output tile ot.
// ------------------------------------------------------------------------------------------
// B32 (33-bin heads): also run this lane group's chain of bin 32 (MzhWMlp::w32) on the hidden units it
// holds, into p32[n]: hidden unit 16ht + 4t + g, ht and t ascending (oracle/mzh_oracle.c linear_head)
// The weight stream goes through a buffer resource: the lane's byte offset sits in one VGPR, the
// fragment / block offset is uniform (SGPR or immediate), so no load costs 64-bit VALU address
// arithmetic (the 64-bit pointer form spent ~13 VALU per two hidden blocks on it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mzw_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ floatx4 mzw_ld4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// rw: the blob's buffer resource (MzhWNet::wbase, made once per kernel: one SGPR quad for every chain)
// Chained form (WS > 0): the rolling buffer is the caller's wst[WS], which arrives holding this chain's
// block 0 (loaded by the previous chain), and the last block's refills load the NEXT chain's block 0
// (fragments 0..WS-1 at byte offset next_soff) instead of the zero pad, so no chain starts on an L2 round trip.
template <int NT, int KB1, int NO, bool OH, bool B32 = false, int WS = 0>
__device__ __forceinline__ void mzw_chain(const MzhWMlp& L, __amdgpu_buffer_rsrc_t rw, const floatx4 (&x)[NT][4],
                                          const float* const (&oh)[NT], floatx4 (&out)[NO][NT], int lane,
                                          float* p32 = nullptr, floatx4* wst = nullptr, int next_soff = 0) {
  constexpr int FR = KB1 + NO;
  static_assert(WS == 0 || WS >= FR, "chained buffer too small");
  const int g = lane >> 4;
  const int vs = 16 * lane, vb = 16 * g;  // byte offsets: the lane's fragment slot, its group's 4 biases
#pragma unroll
  for (int ot = 0; ot < NO; ++ot)
#pragma unroll
    for (int n = 0; n < NT; ++n) out[ot][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  // Rolling weight buffer: slot f holds fragment f of the current hidden block and is refilled
  // with fragment f of the next block as soon as its MFMAs are issued, so every load has the rest
  // of this block's MFMAs (and the next block's up to f) to land.  The scheduling barriers keep
  // the compiler from sinking the refills to their uses.
  floatx4 wloc[WS > 0 ? 1 : FR];
  floatx4* w = WS > 0 ? wst : wloc;
  if constexpr (WS == 0) {
#pragma unroll
    for (int f = 0; f < FR; ++f) w[f] = mzw_ld4(rw, vs, L.soff + f * 1024);
  }
  float a32[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) a32[n] = 0.0f;
#pragma unroll 2
  for (int ht = 0; ht < 16; ++ht) {
    // next block's byte offset (block 16 is the zero pad; chained: the next chain's block 0)
    const int sn = (WS > 0 && ht == 15) ? next_soff : L.soff + (ht + 1) * FR * 1024;
    const floatx4 b = mzw_ld4(rw, vb, L.b1off + 64 * ht);
    floatx4 w32 = {0.f, 0.f, 0.f, 0.f};
    if (B32) w32 = mzw_ld4(rw, vb, L.w32off + 64 * ht);
    floatx4 o[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
      o[n] = OH ? *reinterpret_cast<const floatx4*>(oh[n] + 16 * ht) : floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB1; ++kb) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[kb][t], x[n][kb][t], acc[n], 0, 0, 0);
      w[kb] = mzw_ld4(rw, vs, sn + kb * 1024);
      __builtin_amdgcn_sched_barrier(0);
    }
    floatx4 hid[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[n][i];
        if (OH) v = v + o[n][i];  // one-hot action column (k = 64 + a)
        v = v + b[i];
        hid[n][i] = v > 0.0f ? v : 0.0f;
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int ot = 0; ot < NO; ++ot)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          out[ot][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[KB1 + ot][t], hid[n][t], out[ot][n], 0, 0, 0);
      if (B32) {
#pragma unroll
        for (int n = 0; n < NT; ++n) a32[n] = __builtin_fmaf(hid[n][t], w32[t], a32[n]);
      }
    }
#pragma unroll
    for (int ot = 0; ot < NO; ++ot) w[KB1 + ot] = mzw_ld4(rw, vs, sn + (KB1 + ot) * 1024);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (WS > FR) {  // the next chain's fragments past this chain's slots
#pragma unroll
    for (int f = FR; f < WS; ++f) w[f] = mzw_ld4(rw, vs, next_soff + f * 1024);
  }
  if (B32) {
#pragma unroll
    for (int n = 0; n < NT; ++n) p32[n] = a32[n];
  }
}

template <int NT, int NO>
__device__ __forceinline__ void mzw_bias2(const MzhWMlp& L, __amdgpu_buffer_rsrc_t rw, floatx4 (&out)[NO][NT], int g) {
#pragma unroll
  for (int ot = 0; ot < NO; ++ot) {
    const floatx4 b = mzw_ld4(rw, 16 * g, L.b2off + 64 * ot);
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) out[ot][n][i] = out[ot][n][i] + b[i];
  }
}

// normalize_h_state (networks.py:191-196) of one column: lane group g holds 16 of the 64 units
template <int NT>
__device__ __forceinline__ void mzw_normalize(const floatx4 (&hp)[4][NT], int n, floatx4 (&hn)[NT][4]) {
  float mn = hp[0][n][0], mx = hp[0][n][0];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = hp[ot][n][i];
      mn = __builtin_fminf(v, mn);  // NaN- and -0-free (see mzw_min4g)
      mx = __builtin_fmaxf(v, mx);
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
// NO = 2: bins 0..31 in the tiles, p32 = this lane group's bin-32 chain (mzw_chain B32), b32 its bias
template <int NT, int NO>
__device__ __forceinline__ float mzw_head(const floatx4 (&l)[NO][NT], int n, int lane, float p32 = 0.0f,
                                          float b32 = 0.0f) {
  const int g = lane >> 4;
  if constexpr (NO == 1) {
    return __shfl(l[0][n][0], lane & 15);  // support 1: the raw logit (networks.py:146-148)
  } else {
  static_assert(NO == 2, "33-bin heads: two tiles + the bin-32 chains");
  const bool v8 = g == 0;
  float L[9];
#pragma unroll
  for (int s = 0; s < 8; ++s) L[s] = l[s >> 2][n][s & 3];
  L[8] = mzw_add32(mzw_add16(p32)) + b32;  // ((p0 + p1) + (p2 + p3)) + bias: bin 32 on every group
  float m = L[0];
#pragma unroll
  for (int s = 1; s < 8; ++s) m = __builtin_fmaxf(L[s], m);
  if (v8) m = __builtin_fmaxf(L[8], m);
  m = mzw_max4g(m);
  float e[9];
#pragma unroll
  for (int s = 0; s < 8; ++s) e[s] = mzh_expf_np(L[s] - m);  // arguments <= 0
  e[8] = mzh_expf_np(L[8] - m);  // evaluated on every lane (no divergent branch), kept on group 0
  e[8] = v8 ? e[8] : 0.0f;
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
  t = mzw_add16(t);  // (s0+s1)+(s2+s3) | (s4+s5)+(s6+s7)
  t = mzw_add32(t);
  const float y = 1.0f / t;
  // Markstein quotients, exact while every used exponent argument is >= -65 (t lies in [1, 33], so
  // each numerator is >= e^-65 and each quotient > 2^-100: mzh_fdiv's condition, decided once per
  // lane from the smallest logit); otherwise the wave takes IEEE divisions
  float lmin = L[0];
#pragma unroll
  for (int s = 1; s < 8; ++s) lmin = __builtin_fminf(L[s], lmin);
  if (v8) lmin = __builtin_fminf(L[8], lmin);
  const bool slow = lmin - m < -65.0f;
  float pk[9];
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const float q = e[s] * y;
    pk[s] = __builtin_fmaf(__builtin_fmaf(-q, t, e[s]), y, q);
  }
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
  xs = mzw_add16(xs);
  xs = mzw_add32(xs);
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
    m = __builtin_fmaxf(l[0], m);
    m = __builtin_fmaxf(l[1], m);
  }
  if (ok23) {
    m = __builtin_fmaxf(l[2], m);
    m = __builtin_fmaxf(l[3], m);
  }
  m = mzw_max4g(m);
  // arguments <= 0 on the lanes whose result is used; evaluated on every lane (no divergent branch)
  const float x0 = mzh_expf_np(l[0] - m), x1 = mzh_expf_np(l[1] - m);
  const float x2 = mzh_expf_np(l[2] - m), x3 = mzh_expf_np(l[3] - m);
  const float e0 = ok01 ? x0 : 0.0f, e1 = ok01 ? x1 : 0.0f;
  const float e2 = ok23 ? x2 : 0.0f, e3 = ok23 ? x3 : 0.0f;
  float t = (e0 + e1) + (e2 + e3);
  t = mzw_add16(t);  // group 0: ((s0+s1)+(s2+s3)) + ((s4+s5)+(0+0))
  const float y = 1.0f / t;
  // exactness of the Markstein quotients decided once per lane, as in mzw_head (t lies in [1, 6])
  float lmin = __builtin_inff();
  if (ok01) lmin = __builtin_fminf(__builtin_fminf(l[0], l[1]), lmin);
  if (ok23) lmin = __builtin_fminf(__builtin_fminf(l[2], l[3]), lmin);
  const bool slow = lmin - m < -65.0f;
  auto mdiv = [&](float a) {
    const float q = a * y;
    return __builtin_fmaf(__builtin_fmaf(-q, t, a), y, q);
  };
  floatx4 p;
  p[0] = mdiv(e0);
  p[1] = mdiv(e1);
  p[2] = mdiv(e2);
  p[3] = mdiv(e3);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    p[0] = e0 / t;
    p[1] = e1 / t;
    p[2] = e2 / t;
    p[3] = e3 / t;
  }
  return p;
}

// ---- tree helpers (same arithmetic as mzh_search.hip) ----
// a / b correctly rounded from y = RN(1/b) (Markstein; see mzh_search.hip mzh_div)
__device__ __forceinline__ double mzw_div(double a, double b, double y) {
  const double q = a * y;
  const double r = __builtin_fma(-q, b, a);
  return __builtin_fma(r, y, q);
}
// ucb = fl32(Q) + fl32(U) for one child (node.py:90-123); inv[k] = RN(1/k) (LDS table)
__device__ __forceinline__ float mzw_ucb(int Nc, double Wc, float Rc, double P64, bool p64_semantics, double tnp,
                                         double disc, bool has, double mn, double den, double dinv,
                                         const double* inv, bool exact) {
  // branch-free: both reciprocals in one LDS read, the Q and U chains side by side (for Nc = 0 the
  // Q chain runs on inv[0] = inf and is discarded)
  const double i0 = inv[Nc], i1 = inv[Nc + 1];
  const double v = (double)Rc + disc * mzw_div(Wc, (double)Nc, i0);
  // exact (wave-uniform): IEEE division for a subnormal den (see mzh_tree.h mzh_normalize)
  const double qn = has ? (exact ? (v - mn) / den : mzw_div(v - mn, den, dinv)) : v;
  const float q32 = Nc > 0 ? (float)qn : 0.0f;
  const double w = mzw_div(tnp, (double)(Nc + 1), i1);
  const float u32 = p64_semantics ? (float)(P64 * w) : (float)P64 * (float)w;
  return q32 + u32;
}
// argmax over the 6 children with the reference's tie handling (see mzh_group_pick):
// the 6 children are split over a lane pair (i, i + 32), 3 each: the pair's
// max and its 6-bit argmax mask combine through v_permlane32_swap (max and OR are order-free), so
// both lanes return the same pick and tie bookkeeping
__device__ __forceinline__ int mzw_pick_pair(const float (&u)[3], int half, int tie, int& firstTie, int& extra) {
  float m = u[0];
  m = __builtin_fmaxf(u[1], m);
  m = __builtin_fmaxf(u[2], m);
  float a, b;
  mzw_pair32(m, a, b);
  const float M = __builtin_fmaxf(a, b);
  int mask = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) mask |= (u[j] == M ? 1 : 0) << j;
  mask <<= 3 * half;
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)mask, (unsigned)mask, false, false);
  const int full = (int)(r[0] | r[1]);
  const int cnt = __popc(full);
  const int first = __ffs(full) - 1;
  const bool six = (cnt == MZH_A) & (firstTie == 0);
  extra += ((cnt > 1) & !six) ? 1 : 0;
  firstTie |= six ? 1 : 0;
  return six ? tie : first;
}

// The two waves a SIMD holds drift apart.  Phase-locking them (8-wave workgroups, one barrier per
// simulation before the MLP) was measured 5-10% slower (profiles/r04_experiments.json): each
// simulation then waits for the deepest of 256 roots.
template <int NT, bool REPLAY, bool SUP33>
__global__ __launch_bounds__(MZW_WAVES * 64, 2) void mzh_wave_kernel(MzhWNet net, MzhSearchParams p) {
  constexpr int NOV = SUP33 ? 2 : 1;  // value / reward output tiles (bin 32 of 33: vector chains)
  constexpr int ROOTS = 16 * NT;  // roots per wave
  const float* const noh[NT] = {};  // "no one-hot column" for the chains that take none
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int S = p.S;
  float* ohl = reinterpret_cast<float*>(smem_raw);
  double* table = reinterpret_cast<double*>(smem_raw + sizeof(float) * MZH_A * MZH_F);
  MzwWave<ROOTS>* wsa = reinterpret_cast<MzwWave<ROOTS>*>(smem_raw + mzw_hdr_bytes(S));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar branches)
  const int g = lane >> 4, col = lane & 15;
  const __amdgpu_buffer_rsrc_t rw = mzw_rsrc(net.wbase);

  if (!REPLAY)
    for (int i = tid; i < MZH_A * MZH_F; i += MZW_WAVES * 64) ohl[i] = net.oh[i];
  double* inv = table + (S + 3);
  for (int i = tid; i < S + 3; i += MZW_WAVES * 64) {
    table[i] = i < S + 2 ? p.table[i] : 0.0;
    inv[i] = 1.0 / (double)i;  // IEEE division: correctly rounded
  }
  __syncthreads();  // the only barrier: from here on every wave runs independently
  const int wr0 = (blockIdx.x * MZW_WAVES + wave) * ROOTS;
  if (wr0 >= p.B) return;  // wave-uniform
  MzwWave<ROOTS>& ws = wsa[wave];
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;
  const size_t E = (size_t)p.E;

  // root lanes: lanes rho and rho + 32 (rho < ROOTS) both own root wr0 + rho in the tree phases:
  // selection splits the 6 children between them (3 UCBs per lane), every other tree step runs
  // mirrored on both (same values, same addresses)
  const int rho = lane & 31;
  const int half = lane >> 5;
  const int rroot = wr0 + rho;
  const bool rvalid = rho < ROOTS && rroot < p.B;
  MzwBlock* tb = reinterpret_cast<MzwBlock*>(p.tree) + (size_t)(rvalid ? rroot : 0) * E;
  double mmax = -__builtin_inf(), mmin = __builtin_inf();
  if (rvalid && p.minmax_in) {
    mmax = p.minmax_in[2 * rroot];
    mmin = p.minmax_in[2 * rroot + 1];
  }
  double den = mmax - mmin, dinv = mmax > mmin ? 1.0 / (mmax - mmin) : 0.0;
  int firstTie = 0, extra = 0, steps = 0, rootN = 0, depth = 0, leafE = 0, leafA = 0;
  int lsum = 0;  // p.lockstep_levels: the wave's deepest selection below the root, summed over simulations
  double rootW = 0.0;
  const int tie = (rvalid && p.tie_idx) ? p.tie_idx[rroot] : 0;

  // column lanes: lane (g, col) works on root wr0 + 16n + col of column tile n (MLP phases)
  int croot[NT];
  bool cvalid[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    croot[n] = wr0 + 16 * n + col;
    cvalid[n] = croot[n] < p.B;
  }

  // ---------------- root: initial_inference (mcts.py:49-50) + root.expand (mcts.py:57-69) ----------------
  floatx4 rpi[NT];
  if (!REPLAY) {
    floatx4 hreg[NT][4];  // the root's normalised latent (B-operand order)
    floatx4 x[NT][4];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = 16 * kb + 4 * t + g;
          x[n][kb][t] = (cvalid[n] && k < p.in_dim) ? p.obs[(size_t)croot[n] * p.in_dim + k] : 0.0f;
        }
    floatx4 hp[4][NT];
    switch (net.rep.kb1) {
      case 1: mzw_chain<NT, 1, 4, false>(net.rep, rw, x, noh, hp, lane); break;
      case 2: mzw_chain<NT, 2, 4, false>(net.rep, rw, x, noh, hp, lane); break;
      case 3: mzw_chain<NT, 3, 4, false>(net.rep, rw, x, noh, hp, lane); break;
      default: mzw_chain<NT, 4, 4, false>(net.rep, rw, x, noh, hp, lane); break;
    }
    mzw_bias2<NT, 4>(net.rep, rw, hp, g);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      mzw_normalize<NT>(hp, n, hreg);
      if (cvalid[n]) {
        floatx4* dst = reinterpret_cast<floatx4*>(p.htree + ((size_t)croot[n] * E) * MZH_H) + g;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) dst[4 * kb] = hreg[n][kb];
      }
    }
    floatx4 pl[1][NT];
    mzw_chain<NT, 4, 1, false>(net.pol, rw, hreg, noh, pl, lane);
    mzw_bias2<NT, 1>(net.pol, rw, pl, g);
    floatx4 vl[NOV][NT];
    mzw_chain<NT, 4, NOV, false>(net.val, rw, hreg, noh, vl, lane);  // root value: computed, unused (mcts.py:50)
    (void)vl;
#pragma unroll
    for (int n = 0; n < NT; ++n) rpi[n] = mzw_policy(pl[0][n], lane);
  }
  // root children: prior (Dirichlet-mixed when noised), N = 0, unexpanded
  if (g < 2) {
#pragma unroll
    for (int n = 0; n < NT; ++n)
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
  if (lane < ROOTS) {
#pragma unroll
    for (int c = 0; c < MZH_A; ++c) {
      ws.rW[c][rho] = 0.0;
      ws.rR[c][rho] = 0.0f;
      ws.rN[c][rho] = 0;
      ws.rX[c][rho] = -1;
    }
  }
  mzw_wave_sync();

  int en[NT], an[NT];  // the leaf's parent (expanded index) and move, per column tile
  floatx4 rl[NOV][NT], pl[1][NT], vl[NOV][NT];  // reward / policy / value logits
  float val[NT], rew[NT];
  floatx4 cpi[NT];

  // the four recurrent chains' rolling weight buffer, handed from chain to chain (mzw_chain WS)
  floatx4 wst[8];
  if (!REPLAY) {
#pragma unroll
    for (int f = 0; f < 8; ++f) wst[f] = mzw_ld4(rw, 16 * lane, net.dyn.soff + f * 1024);
  }
  MZH_STAMP_DECL  // diagnostic build: phase stamps (the M phase's are 5-9, see tools/wave_probe.py)
  // select one leaf per root, then hand its parent latent index / move to the column lanes
  // ex: MzhBool<true> = the exact (IEEE-division) normaliser, for a wave where some root's max - min
  // is a non-zero subnormal (caller-given bounds only); chosen once per selection
  auto phase_select = [&](int s, auto ex) {
    (void)s;
    constexpr bool exact = decltype(ex)::value;
    // ---------------- select (mcts.py:75-86; node.py:72-123): one lane per root ----------------
    if (rvalid) {
      const bool has = mmax > mmin;
      float u[3];
      const double tr = table[rootN];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c = 3 * half + j;
        u[j] = mzw_ucb(ws.rN[c][rho], ws.rW[c][rho], ws.rR[c][rho], ws.rP[c][rho], noised || p.np1, tr, disc, has,
                       mmin, den, dinv, inv, exact);
      }
      int pick = mzw_pick_pair(u, half, tie, firstTie, extra);
      int Np = ws.rN[pick][rho], X = ws.rX[pick][rho];
      ws.path[0][rho] = (uint16_t)pick;
      ws.pcW[0][rho] = ws.rW[pick][rho];
      ws.pcR[0][rho] = ws.rR[pick][rho];
      ws.pcN[0][rho] = Np;
      int e = 0, d = 1;
      // 16-root waves (NT = 1) prefetch the children's blocks one level ahead (16,384 roots: 2.66 ->
      // 2.57 ms); at 32 roots per wave the partner wave's MFMA stream already covers the latency
      // (65,536 roots: neutral), so NT = 2 leaves the load queue to the block loads
      constexpr bool kPF = NT == 1;
      int pf0 = 0, pf1 = 0, pf2 = 0;
      while (X >= 0 && d <= S) {  // depth <= s + 1 always; the bound only guards against a corrupt tree
        e = X;
        int nx;
        double Wp;
        float Rp;
        {
          // this lane's half of the block only -- its three children's N|X, R, P and W (5 loads,
          // 60 B, instead of the whole 128-B line on both lanes and a select of each field by half);
          // the picked child's fields come from the lane that holds them over v_permlane32_swap
          // (16,384 roots -1.4%; at 32 roots per wave, once the buffer-load weight stream freed the
          // registers it spilled in round 3: 65,536 roots -0.9%, 262,144 -1.3%)
          const unsigned char* blk = reinterpret_cast<const unsigned char*>(&tb[e]);
          const uint3 hnx = *reinterpret_cast<const uint3*>(blk + 12 * half);
          const uint3 hR = *reinterpret_cast<const uint3*>(blk + 24 + 12 * half);
          const uint3 hP = *reinterpret_cast<const uint3*>(blk + 48 + 12 * half);
          // the W pair at byte 72 + 24 half is only 8-byte aligned: an 8-byte-aligned 16-byte type, so
          // no 16-byte alignment is implied (still one dwordx4: gfx950 global loads need 4-byte alignment)
          typedef unsigned int u32x4_a8 __attribute__((ext_vector_type(4), aligned(8)));
          const u32x4_a8 hW01 = *reinterpret_cast<const u32x4_a8*>(blk + 72 + 24 * half);
          const uint2 hW2 = *reinterpret_cast<const uint2*>(blk + 88 + 24 * half);
          const int hn[3] = {(int)hnx.x, (int)hnx.y, (int)hnx.z};
          const float hr[3] = {__uint_as_float(hR.x), __uint_as_float(hR.y), __uint_as_float(hR.z)};
          const float hp[3] = {__uint_as_float(hP.x), __uint_as_float(hP.y), __uint_as_float(hP.z)};
          const double hw[3] = {__hiloint2double((int)hW01.y, (int)hW01.x), __hiloint2double((int)hW01.w, (int)hW01.z),
                                __hiloint2double((int)hW2.y, (int)hW2.x)};
          if (kPF) {
            asm volatile("" ::"v"(pf0), "v"(pf1), "v"(pf2));
            const int x0 = hn[0] >> 16, x1 = hn[1] >> 16, x2 = hn[2] >> 16;
            pf0 = *reinterpret_cast<const int*>(&tb[x0 >= 0 ? x0 : e]);
            pf1 = *reinterpret_cast<const int*>(&tb[x1 >= 0 ? x1 : e]);
            pf2 = *reinterpret_cast<const int*>(&tb[x2 >= 0 ? x2 : e]);
          }
          const double tn = table[Np];
  #pragma unroll
          for (int j = 0; j < 3; ++j) u[j] = mzw_ucb(hn[j] & 0xFFFF, hw[j], hr[j], (double)hp[j], p.np1, tn, disc, has, mmin, den, dinv, inv, exact);
          pick = mzw_pick_pair(u, half, tie, firstTie, extra);
          // this lane's candidate for the picked slot (valid on the owning half), then the owner's copy
          const int jl = pick - 3 * half;
          int cn = hn[0];
          float cr = hr[0];
          double cw = hw[0];
  #pragma unroll
          for (int q = 1; q < 3; ++q)
            if (jl == q) {
              cn = hn[q];
              cr = hr[q];
              cw = hw[q];
            }
          auto take = [&](unsigned v) {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            // r = {lanes 0-31 value, lanes 32-63 value} on both lanes of the pair
            return pick >= 3 ? r[1] : r[0];
          };
          nx = (int)take((unsigned)cn);
          Rp = __uint_as_float(take(__float_as_uint(cr)));
          const long long wb = __double_as_longlong(cw);
          Wp = __hiloint2double((int)take((unsigned)(wb >> 32)), (int)take((unsigned)(wb & 0xFFFFFFFFll)));
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
      if (kPF) asm volatile("" ::"v"(pf0), "v"(pf1), "v"(pf2));
      depth = d;
      leafE = e;
      leafA = pick;
      steps += d;
    }
    if (p.lockstep_levels) {  // wave-uniform: only when the caller asks for the latency model's input
      int m = rvalid ? depth - 1 : 0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
      lsum += m;
    }
    if (!REPLAY) {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        en[n] = __shfl(leafE, 16 * n + col);
        an[n] = __shfl(leafA, 16 * n + col);
      }
    }
  };

  // M phase: recurrent_inference's four MLPs (networks.py:96-150) as MFMA chains, each head
  // evaluated right after its chain (only scalars stay live)
  auto phase_mlp = [&](int s) {
    if (REPLAY) return;
    // the leaf's parent latent (mcts.py:89-92), stored by an earlier M phase (or the root inference)
    floatx4 x[NT][4];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const floatx4* src = reinterpret_cast<const floatx4*>(p.htree + ((size_t)(cvalid[n] ? croot[n] : 0) * E + en[n]) * MZH_H) + g;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) x[n][kb] = src[4 * kb];
    }
    floatx4 hreg[NT][4];  // the new node's normalised latent
    floatx4 hp[4][NT];
    const float* ohp[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) ohp[n] = ohl + an[n] * MZH_F + 4 * g;
    MZH_STAMP(10);  // latent gather
    mzw_chain<NT, 4, 4, true, false, 8>(net.dyn, rw, x, ohp, hp, lane, nullptr, wst, net.rwd.soff);
    mzw_bias2<NT, 4>(net.dyn, rw, hp, g);  // h' (un-normalised, networks.py:129-138)
    MZH_STAMP(5);
    floatx4 hx[NT][4];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) hx[n][kb] = hp[kb][n];
    float r32[NT], v32[NT];
    mzw_chain<NT, 4, NOV, false, SUP33, 8>(net.rwd, rw, hx, noh, rl, lane, r32, wst, net.pol.soff);  // reward from h' (networks.py:132-135)
    mzw_bias2<NT, NOV>(net.rwd, rw, rl, g);
    MZH_STAMP(6);
#pragma unroll
    for (int n = 0; n < NT; ++n) rew[n] = mzw_head<NT, NOV>(rl, n, lane, SUP33 ? r32[n] : 0.0f, net.rwd.b32);
    MZH_STAMP(11);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      mzw_normalize<NT>(hp, n, hreg);
      if (cvalid[n]) {
        floatx4* dst = reinterpret_cast<floatx4*>(p.htree + ((size_t)croot[n] * E + s + 1) * MZH_H) + g;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) dst[4 * kb] = hreg[n][kb];
      }
    }
    MZH_STAMP(7);
    mzw_chain<NT, 4, 1, false, false, 8>(net.pol, rw, hreg, noh, pl, lane, nullptr, wst, net.val.soff);
    mzw_bias2<NT, 1>(net.pol, rw, pl, g);
#pragma unroll
    for (int n = 0; n < NT; ++n) cpi[n] = mzw_policy(pl[0][n], lane);
    MZH_STAMP(8);
    mzw_chain<NT, 4, NOV, false, SUP33, 8>(net.val, rw, hreg, noh, vl, lane, v32, wst, net.dyn.soff);  // + next dyn block 0
    mzw_bias2<NT, NOV>(net.val, rw, vl, g);
    MZH_STAMP(9);
#pragma unroll
    for (int n = 0; n < NT; ++n) val[n] = mzw_head<NT, NOV>(vl, n, lane, SUP33 ? v32[n] : 0.0f, net.val.b32);
  };

  // the new node's block, then backup (node.py:30-70)
  auto phase_head = [&](int s) {
    if (!REPLAY) {
      // the new node's 6 children (node.py:44-49): N = 0, X = -1, R = 0, P, W = 0.  The whole 128-B
      // line as eight 16-B stores, two per lane group (lane groups 0/1 hold pi[0..3] / pi[4..5]):
      // a line written whole is valid in L2 without a fill from HBM.  Chunk k = bytes 16k..16k+15:
      // 0 nx0-3 | 1 nx4,5 R0,1 | 2 R2-5 | 3 P0-3 | 4 P4,5 W0 | 5 W1,2 | 6 W3,4 | 7 W5 pad
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        if (!cvalid[n]) continue;
        uint4* nb = reinterpret_cast<uint4*>(reinterpret_cast<MzwBlock*>(p.tree) + (size_t)croot[n] * E + s + 1);
        const uint32_t nx = 0xFFFF0000u;  // N = 0, X = -1
        uint4 c0, c1;
        if (g == 0) {
          c0 = make_uint4(nx, nx, nx, nx);
          c1 = make_uint4(__float_as_uint(cpi[n][0]), __float_as_uint(cpi[n][1]), __float_as_uint(cpi[n][2]),
                          __float_as_uint(cpi[n][3]));
        } else if (g == 1) {
          c0 = make_uint4(nx, nx, 0u, 0u);
          c1 = make_uint4(__float_as_uint(cpi[n][0]), __float_as_uint(cpi[n][1]), 0u, 0u);
        } else {
          c0 = make_uint4(0u, 0u, 0u, 0u);
          c1 = c0;
        }
        // g0: chunks 0, 3; g1: chunks 1, 4; g2: chunks 2, 5; g3: chunks 6, 7
        const int k0 = g < 3 ? g : 6, k1 = g < 3 ? g + 3 : 7;
        nb[k0] = c0;
        nb[k1] = c1;
      }
    }
    // ---------------- expand bookkeeping + backup (node.py:30-70): one lane per root ----------------
    if (rvalid) {
      const int enew = s + 1;
      float vv, rr;
      if (REPLAY) {
        const uint4* rec = reinterpret_cast<const uint4*>(p.rp_sim + ((size_t)s * p.B + rroot) * 8);
        const uint4 r0 = rec[0], r1 = rec[1];  // priors 0-3 | priors 4, 5, reward, value
        rr = __uint_as_float(r1.z);
        vv = __uint_as_float(r1.w);
        // the whole 128-B line as eight 16-B stores (see phase_head's fused form)
        uint4* nb = reinterpret_cast<uint4*>(&tb[enew]);
        const uint32_t nx = 0xFFFF0000u;
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
        nb[0] = make_uint4(nx, nx, nx, nx);
        nb[1] = make_uint4(nx, nx, 0u, 0u);
        nb[2] = z;
        nb[3] = r0;
        nb[4] = make_uint4(r1.x, r1.y, 0u, 0u);
        nb[5] = z;
        nb[6] = z;
        nb[7] = z;
      } else {
        // root lane rho is column rho & 15 of tile rho >> 4 (every row of a column holds its scalars)
        vv = val[0];
        rr = rew[0];
#pragma unroll
        for (int n = 1; n < NT; ++n)
          if ((rho >> 4) == n) {
            vv = val[n];
            rr = rew[n];
          }
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
      // path entry j: slot (parent expanded index * 8 + child) and the child's statistics at
      // selection time; entry j - 1 is loaded while entry j is processed
      auto load_lds = [&](int j, int& slot, double& W, float& R, int& N) {
        slot = ws.path[j][rho];
        W = ws.pcW[j][rho];
        R = ws.pcR[j][rho];
        N = ws.pcN[j][rho];
      };
      auto load_hbm = [&](int j, int& slot, double& W, float& R, int& N) {  // depths >= MZW_DC
        slot = p.pathx[(size_t)rroot * E + j];
        const int e = slot >> 3, a = slot & 7;
        W = tb[e].W[a];
        R = tb[e].R[a];
        N = tb[e].nx[a].N;
      };
      int slot;
      double Wj;
      float Rj;
      int Nj;
      // path node j: its statistics (W += v, N += 1), the MinMaxStats candidate, the value chain
      auto node = [&](int j, double& Wn, int& Nn) {
        const double rw = (j == depth - 1) ? (double)rr : (double)Rj;
        Wn = Wj + v;
        Nn = Nj + 1;
        const double q = rw + disc * mzw_div(Wn, (double)Nn, inv[Nn]);  // MinMaxStats input
        lmax = q > lmax ? q : lmax;
        lmin = q < lmin ? q : lmin;
        v = rw + disc * v;
      };
      if (depth - 1 < MZW_DC) load_lds(depth - 1, slot, Wj, Rj, Nj);
      else load_hbm(depth - 1, slot, Wj, Rj, Nj);
      // depths j >= 1 sit in HBM tree blocks (e >= 1), depth 0 is the root's child in LDS (peeled: no
      // per-node branch on where the statistics live); entry j - 1 loaded while node j is processed
      int j = depth - 1;
      auto hbm_node = [&](int jn) {
        const int e = slot >> 3, a = slot & 7;
        double Wn;
        int Nn;
        node(jn, Wn, Nn);
        tb[e].W[a] = Wn;
        tb[e].nx[a].N = (uint16_t)Nn;
      };
      for (; j >= 1; --j) {
        int slot_n, Nj_n;
        double Wj_n;
        float Rj_n;
        if (j - 1 < MZW_DC) load_lds(j - 1, slot_n, Wj_n, Rj_n, Nj_n);
        else load_hbm(j - 1, slot_n, Wj_n, Rj_n, Nj_n);  // paths deeper than the LDS cache (rare)
        hbm_node(j);
        slot = slot_n;
        Wj = Wj_n;
        Rj = Rj_n;
        Nj = Nj_n;
      }
      {  // depth 0: the root's child (path slot = child index, e = 0)
        const int a = slot & 7;
        double Wn;
        int Nn;
        node(0, Wn, Nn);
        ws.rW[a][rho] = Wn;
        ws.rN[a][rho] = Nn;
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
  };

  for (int s = 0; s < S; ++s) {
    MZH_STAMP(4);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(rvalid && mmax > mmin && !(den >= 2.2250738585072014e-308)) != 0, 0))
      phase_select(s, MzhBool<true>{});
    else
      phase_select(s, MzhBool<false>{});
    MZH_STAMP(0);
    // a wave in its matrix phase wins VALU issue arbitration over the co-resident wave's tree work
    // (measured against the tree phases first and against no priorities: profiles/r04_experiments.json)
    __builtin_amdgcn_s_setprio(1);
    phase_mlp(s);
    __builtin_amdgcn_s_setprio(0);
    MZH_STAMP(1);
    phase_head(s);
    MZH_STAMP(2);
    // this simulation's tree stores (other lanes' new-block writes) before the next selection
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }

  // ---------------- results (mcts.py:111-126, 154-176) ----------------
  if (p.lockstep_levels && lane == 0) p.lockstep_levels[blockIdx.x * MZW_WAVES + wave] = lsum;
  if (!rvalid || half) return;
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
      for (int a = 0; a < MZH_A; ++a) v[a] = mzh_pow(v[a], vis[a], ex, p.pow_table);
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

size_t mzh_wave_smem_bytes(int S, int nt) {
  return mzw_hdr_bytes(S) + (nt == 1 ? sizeof(MzwWave<16>) : sizeof(MzwWave<32>)) * MZW_WAVES;
}

template <int NT, bool REPLAY, bool SUP33>
static hipError_t launch_wave_t(const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const size_t smem = mzh_wave_smem_bytes(p.S, NT);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mzh_wave_kernel<NT, REPLAY, SUP33>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int per_wg = MZW_WAVES * 16 * NT;
  const int grid = (p.B + per_wg - 1) / per_wg;
  hipLaunchKernelGGL((mzh_wave_kernel<NT, REPLAY, SUP33>), dim3(grid), dim3(MZW_WAVES * 64), smem, stream, net, p);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_wave_nt(const MzhSearchPlan& pl, const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  if (pl.replay) return pl.sup33 ? launch_wave_t<NT, true, true>(net, p, stream) : launch_wave_t<NT, true, false>(net, p, stream);
  return pl.sup33 ? launch_wave_t<NT, false, true>(net, p, stream) : launch_wave_t<NT, false, false>(net, p, stream);
}

hipError_t mzh_launch_wave_search(const MzhSearchPlan& pl, const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  return pl.nt == 1 ? launch_wave_nt<1>(pl, net, p, stream) : launch_wave_nt<2>(pl, net, p, stream);
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
