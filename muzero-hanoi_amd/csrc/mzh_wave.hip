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

#ifndef MZW_PP
#define MZW_PP 0      // 1: ping-pong schedule across the two waves of each SIMD (8-wave workgroups; measured slower: a lone wave's MFMA stream is not dense enough)
#endif
#ifndef MZW_PRIO
#define MZW_PRIO 0    // ping-pong priority: 0 none, 1 static s_setprio(1) for waves 4-7, 2 M phases
#endif
#ifndef MZW_SPRIO
#define MZW_SPRIO 2   // sequential schedule: 1 static s_setprio(1) for odd workgroups (one of the two
                      // workgroups sharing each SIMD), 2 s_setprio(1) around every M phase
#endif
#ifndef MZW_PPBAR
#define MZW_PPBAR 0   // slot barrier: 0 __syncthreads (drains memory), 1 bare s_barrier
#endif
#ifndef MZW_WAVES
#define MZW_WAVES (MZW_PP ? 8 : 4)  // waves per workgroup
#endif
// NT (template parameter): 16-root MFMA column tiles per wave -- 2 (32 roots) for large batches,
// 1 (16 roots: half the weight reuse) so that mid-size batches still give every SIMD a wave;
// both are built for 2 waves per SIMD (256 VGPRs)
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
#ifndef MZW_ONLYM
#define MZW_ONLYM 0   // DIAGNOSTIC ONLY (wrong results): skip the tree phases, time the MLP phases alone
#endif
#ifndef MZW_XLANE
#define MZW_XLANE 1   // cross-row reductions: 1 = v_permlane16/32_swap, 0 = ds_bpermute shuffles
#endif
#ifndef MZW_RCP
#define MZW_RCP 0     // 1: register reciprocal (rcp + Newton), 0: LDS table of IEEE 1/n
#endif
#ifndef MZW_BKPIPE
#define MZW_BKPIPE 1  // backup: load path entry j-1 while entry j is processed
#endif
#ifndef MZW_SELPF
#define MZW_SELPF 0   // selection: prefetch every child's block (towards L1) one level ahead
#endif
#ifndef MZW_SWP
#define MZW_SWP 0     // MLP chains: layer 2 of hidden block ht-1 issued after layer 1 of block ht (hides the
                      // acc -> ReLU -> layer-2 dependency; same k order, bit-identical)
#endif
#ifndef MZW_PARK
#define MZW_PARK 0    // park the root lanes' tree statistics in LDS across each M phase (3 instead of 6
                      // VGPRs spilled, but neutral: 4.46e8 vs 4.47e8 sims/s over three A/B rounds)
#endif
#ifndef MZW_LAUNDER
#define MZW_LAUNDER 0 // hide each chain's weight base pointer from the optimiser, so the chains' loads of
                      // loop-invariant weight fragments are not hoisted out of the simulation loop (which
                      // kept them live in VGPRs through the tree phases: 256 VGPRs + spills without it)
#endif
// MZW_QC (default 0, mzh_internal.h): cache each child's value R + disc * W / N (fp64, written by
// backup) in the tree block in place of W, so selection skips that division; W moves to the node's
// second cache line (256-B nodes) and reaches backup through the LDS snapshot
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
// MZW_QC: node = the select line (MzwBlock, W[] holding the cached child values) + a line with W
struct __align__(128) MzwNodeQ {
  MzwBlock b;
  double W[6];
  uint32_t pad[20];
};
static_assert(sizeof(MzwNodeQ) == 256, "node layout");
using MzwNode = std::conditional<MZW_QC != 0, MzwNodeQ, MzwBlock>::type;
__device__ __forceinline__ MzwBlock& mzw_blk(MzwBlock* t, int e) { return t[e]; }
__device__ __forceinline__ MzwBlock& mzw_blk(MzwNodeQ* t, int e) { return t[e].b; }
__device__ __forceinline__ double& mzw_wref(MzwBlock* t, int e, int a) { return t[e].W[a]; }
__device__ __forceinline__ double& mzw_wref(MzwNodeQ* t, int e, int a) { return t[e].W[a]; }

// per-wave LDS: the roots' own children (SoA, lane = root: conflict-free) and the path cache
template <int ROOTS>
struct MzwWave {
  double rW[6][ROOTS];
#if MZW_QC
  double rQ[6][ROOTS];  // cached child values of the root's children
#endif
  double rP[6][ROOTS];  // fp64 prior (Dirichlet-mixed or the widened fp32 prior)
  float rR[6][ROOTS];
  int rN[6][ROOTS];
  int rX[6][ROOTS];
  double pcW[MZW_DC][ROOTS];  // chosen child's statistics at each depth (select snapshot)
  float pcR[MZW_DC][ROOTS];
  int pcN[MZW_DC][ROOTS];
  uint16_t path[MZW_DC][ROOTS];  // slot = parent expanded index * 8 + child
#if MZW_PARK
  // a root lane's tree statistics while its wave runs an M phase
  double kd[5][ROOTS];
  int ki[7][ROOTS];
#endif
};

static __host__ __device__ inline size_t mzw_hdr_bytes(int S) {
  size_t b = sizeof(float) * MZH_A * MZH_F + sizeof(double) * (MZW_RCP ? 1 : 2) * (size_t)(S + 3);
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
  if (MZW_XLANE) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  } else {
    const float o = __shfl_xor(v, 16);
    const bool lo = (threadIdx.x & 16) == 0;
    a = lo ? v : o;
    b = lo ? o : v;
  }
}
__device__ __forceinline__ void mzw_pair32(float v, float& a, float& b) {
  if (MZW_XLANE) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  } else {
    const float o = __shfl_xor(v, 32);
    const bool lo = (threadIdx.x & 32) == 0;
    a = lo ? v : o;
    b = lo ? o : v;
  }
}
__device__ __forceinline__ float mzw_max4g(float v) {  // max over the 4 lane groups (rows) of a column
  float a, b;
  mzw_pair16(v, a, b);
  v = a > b ? a : b;
  mzw_pair32(v, a, b);
  return a > b ? a : b;
}
__device__ __forceinline__ float mzw_min4g(float v) {
  float a, b;
  mzw_pair16(v, a, b);
  v = a < b ? a : b;
  mzw_pair32(v, a, b);
  return a < b ? a : b;
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

// RN(1/n) for an integer n >= 1: v_rcp_f64 (not correctly rounded) + two Newton steps.  After the
// first step y1 is within an ulp, so the second step's fma residual 1 - n*y1 is exact and the
// pre-rounding error is ~e^2 < 2^-100, while 1/n is never within 2^-69 (relative) of a rounding
// midpoint for n < 2^16: the single final rounding is RN(1/n), which the Markstein divisions need
// (checked for every n <= 2^20 by mzh_selftest / tests/test_gpu_parity.py).  Replaces a dependent
// LDS table lookup on the select / backup chains.
__device__ __forceinline__ double mzw_rcp_reg(int n) {
  const double d = (double)n;
  const double y0 = __builtin_amdgcn_rcp(d);
  const double y1 = __builtin_fma(y0, __builtin_fma(-d, y0, 1.0), y0);
  return __builtin_fma(y1, __builtin_fma(-d, y1, 1.0), y1);
}
// the search kernel's RN(1/n): LDS table of IEEE 1/n (default) or the register form above
__device__ __forceinline__ double mzw_rcp(int n, const double* inv) { return MZW_RCP ? mzw_rcp_reg(n) : inv[n]; }


// an SGPR pointer the optimiser cannot see through (MZW_LAUNDER)
__device__ __forceinline__ const float4* mzw_opaque(const float4* q) {
  if (MZW_LAUNDER) asm volatile("" : "+s"(q));
  return q;
}

// ------------------------------------------------------------------------------------------
// One MLP (layer1 + bias (+ one-hot column) + ReLU -> layer2, bias2 left to the caller) for the
// wave's 2 column tiles.  x[n][kb] = the B operand of column tile n, k-block kb (lane group g
// holds inputs 16kb + 4t + g, t = 0..3).  out[ot][n]: C registers of output tile ot.
// ------------------------------------------------------------------------------------------
// Software-pipelined form (MZW_SWP): iteration ht issues layer 1 of hidden block ht, then layer 2
// of block ht-1 (its ReLU output computed one iteration earlier), then block ht's ReLU, so the
// MFMA pipe never waits on acc -> bias/ReLU -> layer 2.  Every dot product keeps its k order
// (layer 2 still accumulates block ht-1 before block ht).  Weight slots: w[0..KB1) roll layer-1
// fragments one block ahead; w[KB1..FR) hold the layer-2 fragments of the block whose layer 2 is
// next, refilled right after use; in the last iteration the layer-1 slots take block 15's layer-2
// fragments (instead of the zero pad) so the epilogue's loads were issued a whole layer-1 earlier.
template <int NT, int KB1, int NO, bool OH, bool LAST>
__device__ __forceinline__ void mzw_swp_iter(int ht, const floatx4* S, floatx4 (&w)[KB1 + NO], const float* B1,
                                             const floatx4 (&x)[NT][4], const float* const (&oh)[NT],
                                             floatx4 (&hprev)[NT], floatx4 (&out)[NO][NT]) {
  constexpr int FR = KB1 + NO;
  const floatx4* Sn = S + (ht + 1) * FR * 64;
  const floatx4* Sc = S + ht * FR * 64;
  const floatx4 b = *reinterpret_cast<const floatx4*>(B1 + 16 * ht);
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
    if (!LAST)
      w[kb] = Sn[kb * 64];
    else if (kb < NO)
      w[kb] = Sc[(KB1 + kb) * 64];  // block 15's layer-2 fragment ot = kb, for the epilogue
    if (MZW_PIN) __builtin_amdgcn_sched_barrier(0);
  }
  if (ht > 0) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int ot = 0; ot < NO; ++ot)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          out[ot][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[KB1 + ot][t], hprev[n][t], out[ot][n], 0, 0, 0);
    if (!LAST) {
#pragma unroll
      for (int ot = 0; ot < NO; ++ot) w[KB1 + ot] = Sc[(KB1 + ot) * 64];
    }
  }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = acc[n][i];
      if (OH) v = v + o[n][i];  // one-hot action column (k = 64 + a)
      v = v + b[i];
      hprev[n][i] = v > 0.0f ? v : 0.0f;
    }
  }
  if (MZW_PIN) __builtin_amdgcn_sched_barrier(0);
}

template <int NT, int KB1, int NO, bool OH>
__device__ __forceinline__ void mzw_chain_swp(const MzhWMlp& L, const floatx4 (&x)[NT][4],
                                              const float* const (&oh)[NT], floatx4 (&out)[NO][NT], int lane) {
  constexpr int FR = KB1 + NO;
  const int g = lane >> 4;
  const floatx4* S = reinterpret_cast<const floatx4*>(mzw_opaque(L.s)) + lane;
  const float* B1 = L.b1 + 4 * g;
#pragma unroll
  for (int ot = 0; ot < NO; ++ot)
#pragma unroll
    for (int n = 0; n < NT; ++n) out[ot][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 w[FR];
#pragma unroll
  for (int f = 0; f < FR; ++f) w[f] = S[f * 64];
  floatx4 hprev[NT];
  MZW_UNROLL_PRAGMA
  for (int ht = 0; ht < 15; ++ht) mzw_swp_iter<NT, KB1, NO, OH, false>(ht, S, w, B1, x, oh, hprev, out);
  mzw_swp_iter<NT, KB1, NO, OH, true>(15, S, w, B1, x, oh, hprev, out);
  // epilogue: layer 2 of block 15 (fragments in the layer-1 slots, see mzw_swp_iter)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int ot = 0; ot < NO; ++ot)
#pragma unroll
      for (int n = 0; n < NT; ++n)
        out[ot][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[ot][t], hprev[n][t], out[ot][n], 0, 0, 0);
}

template <int NT, int KB1, int NO, bool OH>
__device__ __forceinline__ void mzw_chain(const MzhWMlp& L, const floatx4 (&x)[NT][4], const float* const (&oh)[NT],
                                          floatx4 (&out)[NO][NT], int lane) {
  if constexpr (MZW_SWP && KB1 >= NO) {
    mzw_chain_swp<NT, KB1, NO, OH>(L, x, oh, out, lane);
    return;
  }
  constexpr int FR = KB1 + NO;
  const int g = lane >> 4;
  const floatx4* S = reinterpret_cast<const floatx4*>(mzw_opaque(L.s)) + lane;
  const float* B1 = L.b1 + 4 * g;
#pragma unroll
  for (int ot = 0; ot < NO; ++ot)
#pragma unroll
    for (int n = 0; n < NT; ++n) out[ot][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  // Rolling weight buffer: slot f holds fragment f of the current hidden block and is refilled
  // with fragment f of the next block as soon as its MFMAs are issued, so every load has the rest
  // of this block's MFMAs (and the next block's up to f) to land.  The scheduling barriers keep
  // the compiler from sinking the refills to their uses.
  floatx4 w[FR];
#pragma unroll
  for (int f = 0; f < FR; ++f) w[f] = S[f * 64];
  MZW_UNROLL_PRAGMA
  for (int ht = 0; ht < 16; ++ht) {
    const floatx4* Sn = S + (ht + 1) * FR * 64;  // block 16 is the zero pad
    const floatx4 b = *reinterpret_cast<const floatx4*>(B1 + 16 * ht);
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
      w[kb] = Sn[kb * 64];
      if (MZW_PIN) __builtin_amdgcn_sched_barrier(0);
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
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int ot = 0; ot < NO; ++ot)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          out[ot][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[KB1 + ot][t], hid[n][t], out[ot][n], 0, 0, 0);
#pragma unroll
    for (int ot = 0; ot < NO; ++ot) w[KB1 + ot] = Sn[(KB1 + ot) * 64];
    if (MZW_PIN) __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NT, int NO>
__device__ __forceinline__ void mzw_bias2(const MzhWMlp& L, floatx4 (&out)[NO][NT], int g) {
#pragma unroll
  for (int ot = 0; ot < NO; ++ot) {
    const floatx4 b = *reinterpret_cast<const floatx4*>(L.b2 + 16 * ot + 4 * g);
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
template <int NT, int NO>
__device__ __forceinline__ float mzw_head(const floatx4 (&l)[NO][NT], int n, int lane) {
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
  t = mzw_add16(t);  // (s0+s1)+(s2+s3) | (s4+s5)+(s6+s7)
  t = mzw_add32(t);
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
  t = mzw_add16(t);  // group 0: ((s0+s1)+(s2+s3)) + ((s4+s5)+(0+0))
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
    const double v = (double)Rc + disc * mzw_div(Wc, (double)Nc, mzw_rcp(Nc, inv));
    q32 = (float)(has ? mzw_div(v - mn, den, dinv) : v);
  }
  const double w = mzw_div(tnp, (double)(Nc + 1), mzw_rcp(Nc + 1, inv));
  const float u32 = p64_semantics ? (float)(P64 * w) : (float)P64 * (float)w;
  return q32 + u32;
}
// the same UCB from a cached child value v = R + disc * W / N (MZW_QC)
__device__ __forceinline__ float mzw_ucbq(int Nc, double v, double P64, bool p64_semantics, double tnp, bool has,
                                          double mn, double den, double dinv, const double* inv) {
  float q32 = 0.0f;
  if (Nc > 0) q32 = (float)(has ? mzw_div(v - mn, den, dinv) : v);
  const double w = mzw_div(tnp, (double)(Nc + 1), mzw_rcp(Nc + 1, inv));
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

template <int NT, bool REPLAY, bool SUP33>
__global__ __launch_bounds__(MZW_WAVES * 64, 8 / MZW_WAVES) void mzh_wave_kernel(MzhWNet net, MzhSearchParams p) {
  constexpr int NOV = SUP33 ? 3 : 1;
  constexpr int ROOTS = 16 * NT;  // roots per wave
  const float* const noh[NT] = {};  // "no one-hot column" for the chains that take none
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int S = p.S;
  float* ohl = reinterpret_cast<float*>(smem_raw);
  double* table = reinterpret_cast<double*>(smem_raw + sizeof(float) * MZH_A * MZH_F);
  MzwWave<ROOTS>* wsa = reinterpret_cast<MzwWave<ROOTS>*>(smem_raw + mzw_hdr_bytes(S));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar branches, s_setprio)
  const int g = lane >> 4, col = lane & 15;

  if (!REPLAY)
    for (int i = tid; i < MZH_A * MZH_F; i += MZW_WAVES * 64) ohl[i] = net.oh[i];
  double* inv = MZW_RCP ? nullptr : table + (S + 3);
  for (int i = tid; i < S + 3; i += MZW_WAVES * 64) {
    table[i] = i < S + 2 ? p.table[i] : 0.0;
    if (!MZW_RCP) inv[i] = 1.0 / (double)i;
  }
  __syncthreads();  // the only barrier: from here on every wave runs independently
  const int wr0 = (blockIdx.x * MZW_WAVES + wave) * ROOTS;
  const bool wactive = wr0 < p.B;  // wave-uniform
  if (!MZW_PP && !wactive) return;  // (ping-pong: idle waves still meet every slot barrier)
  MzwWave<ROOTS>& ws = wsa[wave];
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;
  const size_t E = (size_t)p.E;

  // root lanes: lane rho < 32 owns root wr0 + rho (tree phases)
  const int rho = lane;
  const int rroot = wr0 + rho;
  const bool rvalid = lane < ROOTS && rroot < p.B;
  MzwNode* tb = reinterpret_cast<MzwNode*>(p.tree) + (size_t)(rvalid ? rroot : 0) * E;
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
  int croot[NT];
  bool cvalid[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    croot[n] = wr0 + 16 * n + col;
    cvalid[n] = croot[n] < p.B;
  }


  // ---------------- root: initial_inference (mcts.py:49-50) + root.expand (mcts.py:57-69) ----------------
  floatx4 rpi[NT];
  if (!REPLAY && wactive) {
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
      case 1: mzw_chain<NT, 1, 4, false>(net.rep, x, noh, hp, lane); break;
      case 2: mzw_chain<NT, 2, 4, false>(net.rep, x, noh, hp, lane); break;
      case 3: mzw_chain<NT, 3, 4, false>(net.rep, x, noh, hp, lane); break;
      default: mzw_chain<NT, 4, 4, false>(net.rep, x, noh, hp, lane); break;
    }
    mzw_bias2<NT, 4>(net.rep, hp, g);
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
    mzw_chain<NT, 4, 1, false>(net.pol, hreg, noh, pl, lane);
    mzw_bias2<NT, 1>(net.pol, pl, g);
    floatx4 vl[NOV][NT];
    mzw_chain<NT, 4, NOV, false>(net.val, hreg, noh, vl, lane);  // root value: computed, unused (mcts.py:50)
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
#if MZW_QC
      ws.rQ[c][rho] = 0.0;
#endif
      ws.rR[c][rho] = 0.0f;
      ws.rN[c][rho] = 0;
      ws.rX[c][rho] = -1;
    }
  }
  mzw_wave_sync();

  // ---- per-simulation phases (shared by both schedules below) ----
  int en[NT], an[NT];    // the leaf's parent (expanded index) and move, per column tile
  // heads: evaluated inside the M phase right after their chain (only scalars stay live), or, in
  // the ping-pong schedule, deferred to the T phase with the logits carried across
  constexpr bool HEADS_IN_M = !MZW_PP;
  floatx4 rl[NOV][NT], pl[1][NT], vl[NOV][NT];  // reward / policy / value logits
  float val[NT], rew[NT];
  floatx4 cpi[NT];

  auto mzw_rq = [&](int c) -> double {  // cached value of root child c (MZW_QC)
#if MZW_QC
    return ws.rQ[c][rho];
#else
    (void)c;
    return 0.0;
#endif
  };

  // T-phase part 1: select one leaf per root, then gather its parent latent
  auto phase_select = [&](int s) {
    if (MZW_ONLYM) {  // DIAGNOSTIC ONLY: no tree work (the MLP always expands the root's first child)
      for (int n = 0; n < NT; ++n) en[n] = an[n] = 0;
      return;
    }
    // ---------------- select (mcts.py:75-86; node.py:72-123): one lane per root ----------------
    if (rvalid) {
      const bool has = mmax > mmin;
      float u[6];
      const double tr = table[rootN];
#pragma unroll
      for (int c = 0; c < MZH_A; ++c)
        u[c] = MZW_QC ? mzw_ucbq(ws.rN[c][rho], mzw_rq(c), ws.rP[c][rho], noised || p.np1, tr, has, mmin, den,
                                 dinv, inv)
                      : mzw_ucb(ws.rN[c][rho], ws.rW[c][rho], ws.rR[c][rho], ws.rP[c][rho], noised || p.np1, tr, disc,
                                has, mmin, den, dinv, inv);
      int pick = mzw_pick(u, tie, firstTie, extra);
      int Np = ws.rN[pick][rho], X = ws.rX[pick][rho];
      ws.path[0][rho] = (uint16_t)pick;
      ws.pcW[0][rho] = ws.rW[pick][rho];
      ws.pcR[0][rho] = ws.rR[pick][rho];
      ws.pcN[0][rho] = Np;
      int e = 0, d = 1;
      int pf[6];
      if (MZW_SELPF) {
        // the next level's block is one of the root children's: bring all of them towards L1 now
#pragma unroll
        for (int c = 0; c < MZH_A; ++c) {
          const int xc = ws.rX[c][rho];
          pf[c] = *reinterpret_cast<const int*>(tb + (xc >= 0 ? xc : 0));
        }
      }
      double wpend = 0.0;  // MZW_QC: the chosen child's W (second node line), in flight to pcW[dpend]
      int dpend = -1;
      while (X >= 0 && d <= S) {  // depth <= s + 1 always; the bound only guards against a corrupt tree
        e = X;
        const int4* bp = reinterpret_cast<const int4*>(&mzw_blk(tb, e));
        int dw[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int4 q = bp[k];
          dw[4 * k] = q.x;
          dw[4 * k + 1] = q.y;
          dw[4 * k + 2] = q.z;
          dw[4 * k + 3] = q.w;
        }
        if (MZW_SELPF) {
          // retire the previous prefetches (older than this block's loads: no extra wait), then
          // prefetch this node's children while its UCBs are computed
#pragma unroll
          for (int c = 0; c < MZH_A; ++c) asm volatile("" ::"v"(pf[c]));
#pragma unroll
          for (int c = 0; c < MZH_A; ++c) {
            const int xc = dw[c] >> 16;
            pf[c] = *reinterpret_cast<const int*>(tb + (xc >= 0 ? xc : e));
          }
        }
        double Wc[6];
        float Rc[6];
#pragma unroll
        for (int c = 0; c < MZH_A; ++c) {
          Rc[c] = __int_as_float(dw[6 + c]);
          Wc[c] = __hiloint2double(dw[19 + 2 * c], dw[18 + 2 * c]);  // MZW_QC: the cached child value
          u[c] = MZW_QC ? mzw_ucbq(dw[c] & 0xFFFF, Wc[c], (double)__int_as_float(dw[12 + c]), p.np1, table[Np], has,
                                   mmin, den, dinv, inv)
                        : mzw_ucb(dw[c] & 0xFFFF, Wc[c], Rc[c], (double)__int_as_float(dw[12 + c]), p.np1, table[Np],
                                  disc, has, mmin, den, dinv, inv);
        }
        if (MZW_QC && dpend >= 0) {  // the previous level's W load is older than this block's loads
          ws.pcW[dpend][rho] = wpend;
          dpend = -1;
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
          if (MZW_QC) {
            wpend = mzw_wref(tb, e, pick);
            dpend = d;
          } else {
            ws.pcW[d][rho] = Wp;
          }
          ws.pcR[d][rho] = Rp;
          ws.pcN[d][rho] = Np;
        } else {
          p.pathx[(size_t)rroot * E + d] = slot;
        }
        ++d;
      }
      if (MZW_SELPF) {
#pragma unroll
        for (int c = 0; c < MZH_A; ++c) asm volatile("" ::"v"(pf[c]));
      }
      if (MZW_QC && dpend >= 0) ws.pcW[dpend][rho] = wpend;
      depth = d;
      leafE = e;
      leafA = pick;
      steps += d;
    }
    if (!REPLAY) {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        en[n] = __shfl(leafE, 16 * n + col);
        an[n] = __shfl(leafA, 16 * n + col);
      }
    }
  };

  // M phase: recurrent_inference's four MLPs (networks.py:96-150) as MFMA chains; the heads wait
  // for the T phase so this phase is matrix work only
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
    mzw_chain<NT, 4, 4, true>(net.dyn, x, ohp, hp, lane);
    mzw_bias2<NT, 4>(net.dyn, hp, g);  // h' (un-normalised, networks.py:129-138)
    floatx4 hx[NT][4];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) hx[n][kb] = hp[kb][n];
    mzw_chain<NT, 4, NOV, false>(net.rwd, hx, noh, rl, lane);  // reward from h' (networks.py:132-135)
    mzw_bias2<NT, NOV>(net.rwd, rl, g);
    if (HEADS_IN_M)
#pragma unroll
      for (int n = 0; n < NT; ++n) rew[n] = mzw_head<NT, NOV>(rl, n, lane);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      mzw_normalize<NT>(hp, n, hreg);
      if (cvalid[n]) {
        floatx4* dst = reinterpret_cast<floatx4*>(p.htree + ((size_t)croot[n] * E + s + 1) * MZH_H) + g;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) dst[4 * kb] = hreg[n][kb];
      }
    }
    mzw_chain<NT, 4, 1, false>(net.pol, hreg, noh, pl, lane);
    mzw_bias2<NT, 1>(net.pol, pl, g);
    if (HEADS_IN_M)
#pragma unroll
      for (int n = 0; n < NT; ++n) cpi[n] = mzw_policy(pl[0][n], lane);
    mzw_chain<NT, 4, NOV, false>(net.val, hreg, noh, vl, lane);
    mzw_bias2<NT, NOV>(net.val, vl, g);
    if (HEADS_IN_M)
#pragma unroll
      for (int n = 0; n < NT; ++n) val[n] = mzw_head<NT, NOV>(vl, n, lane);
  };

  // T-phase part 0: heads of simulation s, the new node's block, backup (node.py:30-70)
  auto phase_head = [&](int s) {
    if (MZW_ONLYM) return;  // DIAGNOSTIC ONLY
    if (!REPLAY) {
      if (!HEADS_IN_M)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          rew[n] = mzw_head<NT, NOV>(rl, n, lane);
          cpi[n] = mzw_policy(pl[0][n], lane);
          val[n] = mzw_head<NT, NOV>(vl, n, lane);
        }
      // the new node's 6 children (node.py:44-49): lane groups 0/1 hold pi[0..3] / pi[4..5]
      if (g < 2) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          if (!cvalid[n]) continue;
          MzwNode* nn = reinterpret_cast<MzwNode*>(p.tree) + (size_t)croot[n] * E;
          MzwBlock* nb = &mzw_blk(nn, s + 1);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = 4 * g + i;
            if (c < MZH_A) {
              *reinterpret_cast<uint32_t*>(&nb->nx[c]) = 0xFFFF0000u;  // N = 0, X = -1
              nb->R[c] = 0.0f;
              nb->P[c] = cpi[n][i];
              nb->W[c] = 0.0;
              if (MZW_QC) mzw_wref(nn, s + 1, c) = 0.0;
            }
          }
        }
      }
    }
    // ---------------- expand bookkeeping + backup (node.py:30-70): one lane per root ----------------
    if (rvalid) {
      const int enew = s + 1;
      float vv, rr;
      if (REPLAY) {
        vv = p.rp_value[(size_t)rroot * S + s];
        rr = p.rp_reward[(size_t)rroot * S + s];
        MzwBlock* nb = &mzw_blk(tb, enew);
#pragma unroll
        for (int c = 0; c < MZH_A; ++c) {
          *reinterpret_cast<uint32_t*>(&nb->nx[c]) = 0xFFFF0000u;
          nb->R[c] = 0.0f;
          nb->P[c] = p.rp_pi[((size_t)rroot * S + s) * MZH_A + c];
          nb->W[c] = 0.0;
          if (MZW_QC) mzw_wref(tb, enew, c) = 0.0;
        }
      } else {
        // root lane rho is column rho & 15 of tile rho >> 4 (every row of a column holds its scalars)
        vv = val[0];
        rr = rew[0];
#pragma unroll
        for (int n = 1; n < NT; ++n)
          if ((lane >> 4) == n) {
            vv = val[n];
            rr = rew[n];
          }
      }
      if (leafE == 0) {
        ws.rX[leafA][rho] = enew;
        ws.rR[leafA][rho] = rr;
      } else {
        mzw_blk(tb, leafE).nx[leafA].X = (int16_t)enew;
        mzw_blk(tb, leafE).R[leafA] = rr;
      }
      double v = (double)vv;
      double lmax = -__builtin_inf(), lmin = __builtin_inf();
      // path entry j: slot (parent expanded index * 8 + child) and the child's statistics at
      // selection time; entry j - 1 is loaded while entry j is processed
      auto load_entry = [&](int j, int& slot, double& W, float& R, int& N) {
        if (j < MZW_DC) {
          slot = ws.path[j][rho];
          W = ws.pcW[j][rho];
          R = ws.pcR[j][rho];
          N = ws.pcN[j][rho];
        } else {
          slot = p.pathx[(size_t)rroot * E + j];
          const int e = slot >> 3, a = slot & 7;
          W = mzw_wref(tb, e, a);
          R = mzw_blk(tb, e).R[a];
          N = mzw_blk(tb, e).nx[a].N;
        }
      };
      int slot;
      double Wj;
      float Rj;
      int Nj;
      if (MZW_BKPIPE) load_entry(depth - 1, slot, Wj, Rj, Nj);
      for (int j = depth - 1; j >= 0; --j) {
        int slot_n = 0, Nj_n = 0;
        double Wj_n = 0.0;
        float Rj_n = 0.0f;
        if (MZW_BKPIPE && j > 0) load_entry(j - 1, slot_n, Wj_n, Rj_n, Nj_n);
        if (!MZW_BKPIPE) load_entry(j, slot, Wj, Rj, Nj);
        const int e = slot >> 3, a = slot & 7;
        const double rw = (j == depth - 1) ? (double)rr : (double)Rj;
        const double Wn = Wj + v;
        const int Nn = Nj + 1;
        // the child's value after this backup: MinMaxStats input, and (MZW_QC) the cached value its
        // next selection reads -- the same operations as mzw_ucb's v
        const double q = rw + disc * mzw_div(Wn, (double)Nn, mzw_rcp(Nn, inv));
        if (e == 0) {
          ws.rW[a][rho] = Wn;
          ws.rN[a][rho] = Nn;
#if MZW_QC
          ws.rQ[a][rho] = q;
#endif
        } else {
          mzw_wref(tb, e, a) = Wn;
          mzw_blk(tb, e).nx[a].N = (uint16_t)Nn;
          if (MZW_QC) mzw_blk(tb, e).W[a] = q;
        }
        lmax = q > lmax ? q : lmax;
        lmin = q < lmin ? q : lmin;
        v = rw + disc * v;
        slot = slot_n;
        Wj = Wj_n;
        Rj = Rj_n;
        Nj = Nj_n;
      }
      rootW = rootW + v;
      rootN = rootN + 1;
      const double q = 0.0 + disc * mzw_div(rootW, (double)rootN, mzw_rcp(rootN, inv));  // root rwd = 0.0
      lmax = q > lmax ? q : lmax;
      lmin = q < lmin ? q : lmin;
      mmax = lmax > mmax ? lmax : mmax;
      mmin = lmin < mmin ? lmin : mmin;
      den = mmax - mmin;
      dinv = mmax > mmin ? 1.0 / (mmax - mmin) : 0.0;
    }
  };

  // MZW_PARK: the root lanes' statistics go to LDS before the M phase and come back after it; the
  // compiler barrier between makes the reloads real, so none of these values is live (in VGPRs)
  // across the MLP chains
  auto park = [&]() {
#if MZW_PARK
    if (lane < ROOTS) {
      ws.kd[0][rho] = mmax;
      ws.kd[1][rho] = mmin;
      ws.kd[2][rho] = den;
      ws.kd[3][rho] = dinv;
      ws.kd[4][rho] = rootW;
      ws.ki[0][rho] = rootN;
      ws.ki[1][rho] = firstTie;
      ws.ki[2][rho] = extra;
      ws.ki[3][rho] = steps;
      ws.ki[4][rho] = depth;
      ws.ki[5][rho] = leafE;
      ws.ki[6][rho] = leafA;
    }
    asm volatile("" ::: "memory");
#endif
  };
  auto unpark = [&]() {
#if MZW_PARK
    asm volatile("" ::: "memory");
    if (lane < ROOTS) {
      mmax = ws.kd[0][rho];
      mmin = ws.kd[1][rho];
      den = ws.kd[2][rho];
      dinv = ws.kd[3][rho];
      rootW = ws.kd[4][rho];
      rootN = ws.ki[0][rho];
      firstTie = ws.ki[1][rho];
      extra = ws.ki[2][rho];
      steps = ws.ki[3][rho];
      depth = ws.ki[4][rho];
      leafE = ws.ki[5][rho];
      leafA = ws.ki[6][rho];
    }
#endif
  };

  MZH_STAMP_DECL
  if (!MZW_PP) {
    if (MZW_SPRIO == 1 && (blockIdx.x & 1)) __builtin_amdgcn_s_setprio(1);
    for (int s = 0; s < S; ++s) {
      MZH_STAMP(4);
      phase_select(s);
      MZH_STAMP(0);
      if (MZW_PARK) park();
      if (MZW_SPRIO == 2) __builtin_amdgcn_s_setprio(1);
      phase_mlp(s);
      if (MZW_SPRIO == 2) __builtin_amdgcn_s_setprio(0);
      if (MZW_PARK) unpark();
      MZH_STAMP(1);
      phase_head(s);
      MZH_STAMP(2);
      // this simulation's tree stores (other lanes' new-block writes) before the next selection
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
    }
  } else {
    // Ping-pong: waves w and w + 4 share a SIMD.  The second half runs one slot behind the first,
    // so in every slot one wave of each SIMD is in an M phase (matrix pipe) while its partner is
    // in a T phase (heads, backup, selection: latency-bound L2 / LDS / fp64 work).  A wave's
    // sequence is T0 = select(0), M0, T1 = head(0) + select(1), M1, ..., M(S-1), TS = head(S-1).
    const int lag = wave >= MZW_WAVES / 2 ? 1 : 0;
    if (MZW_PRIO == 1 && lag) __builtin_amdgcn_s_setprio(1);  // the younger half (guide: static priority)
    for (int k = 0; k < 2 * S + 2; ++k) {
      const int kk = k - lag;
      if (wactive && kk >= 0 && kk <= 2 * S) {
        if ((kk & 1) == 0) {
          const int j = kk >> 1;
          if (j >= 1) phase_head(j - 1);
          MZH_STAMP(2);
          if (j < S) phase_select(j);
          MZH_STAMP(0);
        } else {
          if (MZW_PRIO == 2) __builtin_amdgcn_s_setprio(1);  // matrix phase wins VALU arbitration
          phase_mlp(kk >> 1);
          if (MZW_PRIO == 2) __builtin_amdgcn_s_setprio(0);
          MZH_STAMP(1);
        }
      }
      // slot boundary; the same wave's stores are ordered for the next phase either way
      if (MZW_PPBAR) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
        __syncthreads();
      }
      MZH_STAMP(3);
    }
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

// mzh_selftest(MZH_SELFTEST_RCP): mzw_rcp(n) == IEEE 1.0 / n for every n in [1, nmax]
__global__ void mzw_rcp_check_kernel(int nmax, int32_t* bad) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (n <= nmax && mzw_rcp_reg(n) != 1.0 / (double)n) atomicAdd(bad, 1);
}
hipError_t mzh_launch_rcp_check(int nmax, int32_t* bad, hipStream_t stream) {
  hipLaunchKernelGGL(mzw_rcp_check_kernel, dim3((nmax + 255) / 256), dim3(256), 0, stream, nmax, bad);
  return hipGetLastError();
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
static hipError_t launch_wave_nt(bool replay, const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const bool sup33 = net.support == 33;
  if (replay) return sup33 ? launch_wave_t<NT, true, true>(net, p, stream) : launch_wave_t<NT, true, false>(net, p, stream);
  return sup33 ? launch_wave_t<NT, false, true>(net, p, stream) : launch_wave_t<NT, false, false>(net, p, stream);
}

hipError_t mzh_launch_wave_search(int nt, bool replay, const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream) {
  return nt == 1 ? launch_wave_nt<1>(replay, net, p, stream) : launch_wave_nt<2>(replay, net, p, stream);
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
