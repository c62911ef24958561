// mzh_device.h -- device-side building blocks for libmzh (gfx950 / CDNA4).
//
// Numerics contract (shared with the CPU oracle, oracle/mzh_oracle.c, which restates the same
// algorithms independently): built with -ffp-contract=off, so
//   * every dot product is a k-ordered fp32 FMA chain from 0 (exactly what
//     v_mfma_f32_16x16x4_f32 accumulates), the bias added afterwards;
//   * softmax uses mzh_expf (Cody-Waite + degree-6 polynomial, explicit fmaf);
//   * the signed-parabolic transform follows networks.py:186-189 op by op in fp32 with the
//     python scalars folded exactly as the reference folds them;
//   * tree statistics are fp64 in MCTS/node.py's operation order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MZH_A 6
#define MZH_H 64
#define MZH_F 256
#define MZH_WAVE 64
// waves per cooperative workgroup (an 8-wave schedule, two per SIMD, measured +3% at 6-8k roots with
// 32-row tiles and -14% at <= 4k roots with 16-row tiles: not kept)
#define MZH_WAVES 4
#define MZH_THREADS (64 * MZH_WAVES)

typedef float floatx4 __attribute__((ext_vector_type(4)));

// a compile-time bool carried by value (selects a specialised copy of a generic lambda)
template <bool B>
struct MzhBool {
  static constexpr bool value = B;
};

// ------------------------------------------------------------------------------------------
// Diagnostic phase stamps (only in the -DMZH_STAMPS build, libmzh_diag.so; never in libmzh.so).
// Lane 0 of every wave accumulates s_memtime deltas per phase into mzh_stamp_acc[wave][phase].
// ------------------------------------------------------------------------------------------
#define MZH_NSTAMP 32
#ifdef MZH_STAMPS
__device__ unsigned long long mzh_stamp_acc[8][MZH_NSTAMP];
#define MZH_STAMP_DECL unsigned long long mzh_t_prev = __builtin_amdgcn_s_memtime();
#define MZH_STAMP(ph)                                                                       \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
    if ((threadIdx.x & 63) == 0 && blockIdx.x == 0)                                         \
      atomicAdd(&mzh_stamp_acc[threadIdx.x >> 6][ph], t_ - mzh_t_prev);                      \
    mzh_t_prev = t_;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                      \
  } while (0)
// register-accumulated stamps for divergent loops (flushed once by the first active lane)
#define MZH_LSTAMP_DECL                                         \
  unsigned long long mzh_lt_prev = __builtin_amdgcn_s_memtime(); \
  unsigned long long mzh_lacc[5] = {0, 0, 0, 0, 0};
#define MZH_LSTAMP(i)                                         \
  do {                                                        \
    __builtin_amdgcn_sched_barrier(0);                        \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    mzh_lacc[i] += t_ - mzh_lt_prev;                          \
    mzh_lt_prev = t_;                                         \
    __builtin_amdgcn_sched_barrier(0);                        \
  } while (0)
#define MZH_LSTAMP_COUNT() (mzh_lacc[4] += 1)
#define MZH_LSTAMP_FLUSH(base)                                                                  \
  do {                                                                                          \
    if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1 && blockIdx.x == 0)        \
      for (int i_ = 0; i_ < 5; ++i_) atomicAdd(&mzh_stamp_acc[threadIdx.x >> 6][(base) + i_], mzh_lacc[i_]); \
  } while (0)
#else
#define MZH_STAMP_DECL
#define MZH_STAMP(ph) do {} while (0)
#define MZH_LSTAMP_DECL
#define MZH_LSTAMP(i) do {} while (0)
#define MZH_LSTAMP_COUNT() do {} while (0)
#define MZH_LSTAMP_FLUSH(base) do {} while (0)
#endif

// ------------------------------------------------------------------------------------------
// fp32 math (networks.py:152-196)
// ------------------------------------------------------------------------------------------
// Branch-free: the polynomial runs for every lane and the range checks select the result (a
// divergent branch per exponential costs an exec-mask round trip; outside the range the computed
// value is discarded), so the result is the same as testing first
__device__ __forceinline__ float mzh_expf(float x) {
  float n = __builtin_rintf(x * 1.44269502162933349609375f);
  float r = __builtin_fmaf(n, -0.693359375f, x);
  r = __builtin_fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = __builtin_fmaf(p, r, 1.3981999507e-3f);
  p = __builtin_fmaf(p, r, 8.3334519073e-3f);
  p = __builtin_fmaf(p, r, 4.1665795894e-2f);
  p = __builtin_fmaf(p, r, 1.6666665459e-1f);
  p = __builtin_fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  p = __builtin_fmaf(p, r2, r);
  p = p + 1.0f;
  int ni = (int)n;
  const float e = p * __int_as_float((ni + 127) << 23);
  return x < -87.0f ? 0.0f : (x > 88.0f ? __builtin_inff() : e);
}

// mzh_expf for x <= 0 (softmax arguments l - max): the overflow check dropped
__device__ __forceinline__ float mzh_expf_np(float x) {
  float n = __builtin_rintf(x * 1.44269502162933349609375f);
  float r = __builtin_fmaf(n, -0.693359375f, x);
  r = __builtin_fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = __builtin_fmaf(p, r, 1.3981999507e-3f);
  p = __builtin_fmaf(p, r, 8.3334519073e-3f);
  p = __builtin_fmaf(p, r, 4.1665795894e-2f);
  p = __builtin_fmaf(p, r, 1.6666665459e-1f);
  p = __builtin_fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  p = __builtin_fmaf(p, r2, r);
  p = p + 1.0f;
  int ni = (int)n;
  const float e = p * __int_as_float((ni + 127) << 23);
  return x < -87.0f ? 0.0f : e;
}

// _signed_parabolic of two independent values as one packed chain (v_pk_* ops; the same
// operations per element as mzh_signed_parabolic below, so the same results)
typedef float mzh_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ mzh_f2 mzh_signed_parabolic2(mzh_f2 x) {
  const mzh_f2 a = {__builtin_fabsf(x.x), __builtin_fabsf(x.y)};
  mzh_f2 t = 1.00100004673004150390625f + a;
  t = 0.0040000001899898052215576171875f * t;
  t = 1.0f + t;
  t = mzh_f2{__builtin_sqrtf(t.x), __builtin_sqrtf(t.y)};
  t = t * 0.5f;  // t / 2.0f: exact
  {
    const mzh_f2 b = 0.001000000047497451305389404296875f, y = 0x1.f3fffep+9f;
    const mzh_f2 q = t * y;
    const mzh_f2 r = __builtin_elementwise_fma(-q, b, t);
    t = __builtin_elementwise_fma(r, y, q);
  }
  const mzh_f2 z = t - 500.0f;
  const mzh_f2 sg = {x.x > 0.0f ? 1.0f : (x.x < 0.0f ? -1.0f : 0.0f), x.y > 0.0f ? 1.0f : (x.y < 0.0f ? -1.0f : 0.0f)};
  return sg * (z * z - 1.0f);
}

// _signed_parabolic (networks.py:186-189)
__device__ __forceinline__ float mzh_signed_parabolic(float x) {
  float a = __builtin_fabsf(x);
  float t = 1.00100004673004150390625f + a;
  t = 0.0040000001899898052215576171875f * t;
  t = 1.0f + t;
  t = __builtin_sqrtf(t);
  t = t / 2.0f;
  {  // t / 0.001f (t >= 0.5 here) by Markstein from y = RN(1/0.001f): equal to the IEEE quotient
     // for every float t >= 0.5 whose quotient is finite (checked exhaustively, tools/markstein_c.c)
    const float b = 0.001000000047497451305389404296875f, y = 0x1.f3fffep+9f;
    const float q = t * y;
    const float r = __builtin_fmaf(-q, b, t);
    t = __builtin_fmaf(r, y, q);
  }
  float z = t - 500.0f;
  float sg = x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f);
  return sg * (z * z - 1.0f);
}

// ------------------------------------------------------------------------------------------
// 8-lane DPP reductions (aligned groups of 8 lanes; no LDS crossbar).  Steps: quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror (lane i <-> 7-i).  Every source lane lies in the
// reading lane's own 8-lane group, whose lanes are always active together, so bound_ctrl = 1 changes
// nothing but lets the compiler fold each move into its consumer (v_add_f32_dpp, v_or_b32_dpp).  Every lane of the group ends
// with the same bits: IEEE add/max are commutative, so the sum is exactly
// ((s0+s1)+(s2+s3)) + ((s4+s5)+(s6+s7)) on every lane -- the order oracle/mzh_oracle.c uses.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float mzh_dpp_f(float v, int ctrl_sel) {
  switch (ctrl_sel) {
    case 0: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
    case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
    default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));
  }
}
__device__ __forceinline__ float mzh_max8(float v) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float t = mzh_dpp_f(v, i);
    v = t > v ? t : v;
  }
  return v;
}
// max over the group for NaN-free values (UCB scores: finite or -inf): one v_max_f32_dpp per step
// instead of move + compare + select (fmaxf would add canonicalising maxes in IEEE mode).  A max of
// +0 and -0 may return either zero; the callers only compare for equality, where they are equal.
__device__ __forceinline__ float mzh_max8_nonan(float v) {
  float a, b, c;
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a) : "v"(v));
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "=v"(b) : "v"(a));
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf" : "=v"(c) : "v"(b));
  return c;
}
// NaN- and -0-free operands (the latent normalisation's raw units: an FMA chain from +0 plus a bias
// never rounds to -0): v_min / v_max, no compare + select, no canonicalising of LDS-loaded operands
__device__ __forceinline__ float mzh_vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float mzh_vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float mzh_min8_nonan(float v) {
  float a, b, c;
  asm volatile("s_nop 1\n\tv_min_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a) : "v"(v));
  asm volatile("s_nop 1\n\tv_min_f32_dpp %0, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "=v"(b) : "v"(a));
  asm volatile("s_nop 1\n\tv_min_f32_dpp %0, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf" : "=v"(c) : "v"(b));
  return c;
}
__device__ __forceinline__ float mzh_min8(float v) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float t = mzh_dpp_f(v, i);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ float mzh_sum8(float v) {
#pragma unroll
  for (int i = 0; i < 3; ++i) v = v + mzh_dpp_f(v, i);
  return v;
}

// the value of the one lane of an aligned 8-lane group with `sel` set, on every lane of the group
// (an OR over the DPP tree: three VALU steps instead of a ds_bpermute round trip)
__device__ __forceinline__ int mzh_group_take(int v, bool sel) {
  int x = sel ? v : 0;
  x |= __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);
  x |= __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);
  x |= __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true);
  return x;
}

__device__ __forceinline__ double mzh_dpp_d(double v, int ctrl_sel) {
  const long long b = __double_as_longlong(v);
  const int lo = (int)(b & 0xFFFFFFFFll), hi = (int)(b >> 32);
  int l2, h2;
  switch (ctrl_sel) {
    case 0:
      l2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, true);
      h2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, true);
      break;
    case 1:
      l2 = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, true);
      h2 = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, true);
      break;
    default:
      l2 = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, true);
      h2 = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, true);
      break;
  }
  return __longlong_as_double(((long long)h2 << 32) | (unsigned)l2);
}
// max / min over an aligned 8-lane group (exact: order-free)
__device__ __forceinline__ void mzh_maxmin8d(double& mx, double& mn) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double tx = mzh_dpp_d(mx, i), tn = mzh_dpp_d(mn, i);
    mx = tx > mx ? tx : mx;
    mn = tn < mn ? tn : mn;
  }
}

// logits_to_transformed_expected_value (networks.py:152-184); logits in LDS
__device__ inline float mzh_logits_to_value(const float* l, int support) {
  if (support == 1) return l[0];
  float m = l[0];
  for (int i = 1; i < support; ++i) m = l[i] > m ? l[i] : m;
  float e[33];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 33; ++i) {
    e[i] = mzh_expf(l[i] - m);
    s = s + e[i];
  }
  const int half = 16;
  float x = 0.0f;
#pragma unroll
  for (int k = 0; k < 33; ++k) {
    float p = e[k] / s;
    float prod = p * (float)(k - half);
    x = x + prod;
  }
  return mzh_signed_parabolic(x);
}

__device__ inline void mzh_softmax6(const float* l, float* p) {
  float m = l[0];
#pragma unroll
  for (int i = 1; i < MZH_A; ++i) m = l[i] > m ? l[i] : m;
  float e[MZH_A];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < MZH_A; ++i) {
    e[i] = mzh_expf(l[i] - m);
    s = s + e[i];
  }
#pragma unroll
  for (int i = 0; i < MZH_A; ++i) p[i] = e[i] / s;
}

// ------------------------------------------------------------------------------------------
// Packed network (built by mzh_load_weights).  Each nn.Linear [N][K] is stored as MFMA B
// fragments: tile nt (16 output columns) x k-block kb (16 inputs) x lane -> one float4 holding
// the lane's B values for the 4 consecutive k-steps of the block:
//     W4[(nt*KB + kb)*64 + lane][j] = W[16nt + (lane&15)][16kb + 4j + (lane>>4)]
// so one global_load_dwordx4 per lane (1 KiB per wave, coalesced) feeds 4 MFMAs.
// N and K are zero-padded to multiples of 16 (padding at the END of k keeps the FMA chain).
// ------------------------------------------------------------------------------------------
struct MzhLayer {
  const float4* w;  // [NT][KB][64]
  const float* b;   // [16*NT]
  int kb, nt;
  int woff, boff;  // byte offsets of w and b in the packed weight blob (MzhNet::wbase)
};

// Support 33: rwd2 / val2 hold bins 0..31 (two 16-row tiles); bin 32 -- which would cost a third
// tile 15/16 padding -- is computed with vector FMAs as four k-ordered chains over k = g, g + 4, ...
// (g = 0..3) combined ((p0 + p1) + (p2 + p3)), bias after (oracle/mzh_oracle.c linear_head).
// rwd32 / val32: [16 blocks b][4 g] float4 {W[32][16b + g], W[32][16b + 4 + g], W[32][16b + 8 + g],
// W[32][16b + 12 + g]}: the weights of chain g in its order (shared with the wave kernel, MzhWMlp::w32)
struct MzhNet {
  MzhLayer rep0, rep2, dyn0, dyn2, rwd0, rwd2, pol0, pol2, val0, val2;
  const float* wbase;  // the packed weight blob every layer lives in (one buffer resource for all chunks)
  const float* dyn0_onehot;  // [6][256]: dynamic_net.0.weight[:, 64 + a]
  const float4 *rwd32, *val32;
  float rwd32b, val32b;
  int support;               // 33 or 1
  int in_dim;                // 3N
};

// ------------------------------------------------------------------------------------------
// LDS layout of the MLP block for R roots (R = 16 * MT).  Buffers read as an MFMA A operand (x,
// hraw, hid*) hold each row's units in *k-block order*: inside every 16-unit block, position
// 4g + j holds unit 4j + g (mzh_kpos, an involution), so the lane (row r, k-group g) of a
// 16x16x4 chain finds its four k-steps' operands of one k-block as one aligned float4: one
// ds_read_b128 per row tile and k-block (one-wave-per-SIMD LDS reads run at full rate only in
// the 128-bit form).  Row strides 4 (mod 64) dwords: at most 2-way bank sharing for those reads,
// conflict-free ds_write_b32 of the C fragments.  Logit buffers keep natural order.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int mzh_kpos(int k) { return (k & ~15) | ((k & 3) << 2) | ((k >> 2) & 3); }
#define MZH_LD64 68
#define MZH_LD256 260
#define MZH_LDPOL 16
#define MZH_LDSUP 40

template <int R>
struct MlpSmem {
  float x[R * MZH_LD64];      // input: obs (initial) / parent latent (recurrent) / normalised h
  float hraw[R * MZH_LD64];   // un-normalised latent (dynamics / representation output)
  float hidR[R * MZH_LD256];  // reward-head hidden
  float hidP[R * MZH_LD256];  // dynamics / policy hidden
  float hidV[R * MZH_LD256];  // value hidden
  float lpol[R * MZH_LDPOL];  // policy logits
  float lval[R * MZH_LDSUP];  // value logits
  float lrwd[R * MZH_LDSUP];  // reward logits
  float w32[2 * 256];         // bin 32 of the 33-bin reward / value heads: rwd32 | val32 packing (mzh_w32_fill)
  float pi[R * 8];
  float value[R];
  float reward[R];
  int act[R];
};

struct MzhJob {
  const float* A;  // LDS, row stride lda
  const float4* W; // packed tile
  float* out;      // LDS, row stride ldo
  const float* bias;
  int lda, ldo, col0, relu;
};

__device__ __forceinline__ MzhJob mzh_job(const float* A, int lda, const MzhLayer& L, int nt, float* out,
                                          int ldo, int relu) {
  MzhJob j;
  j.A = A;
  j.lda = lda;
  j.W = L.w + (size_t)nt * L.kb * 64;
  j.out = out;
  j.ldo = ldo;
  j.bias = L.b;
  j.col0 = nt * 16;
  j.relu = relu;
  return j;
}

// NJ output tiles (jobs) x MT row tiles, all with KB k-blocks, computed by one wave.
// onehot (nullable): dynamics first layer one-hot columns [6][256], indexed by act[row].
template <int MT, int NJ>
__device__ __forceinline__ void mzh_run_jobs(const MzhJob* jobs, int KB, const float* onehot, const int* act,
                                             int lane) {
  const int r = lane & 15, g = lane >> 4;
  floatx4 acc[NJ][MT];
#pragma unroll
  for (int q = 0; q < NJ; ++q)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[q][m] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 bc[NJ], bn[NJ];
#pragma unroll
  for (int q = 0; q < NJ; ++q) {
    float4 t = jobs[q].W[lane];
    bc[q] = floatx4{t.x, t.y, t.z, t.w};
  }
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 1 < KB) {
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
        float4 t = jobs[q].W[(kb + 1) * 64 + lane];
        bn[q] = floatx4{t.x, t.y, t.z, t.w};
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kp = kb * 16 + g * 4 + j;  // position of k = 16kb + 4j + g (k-block order)
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          float a = jobs[q].A[(m * 16 + r) * jobs[q].lda + kp];
          acc[q][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bc[q][j], acc[q][m], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NJ; ++q) bc[q] = bn[q];
  }
  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + i
#pragma unroll
  for (int q = 0; q < NJ; ++q) {
    const int col = jobs[q].col0 + r;
    const float bias = jobs[q].bias[col];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m * 16 + g * 4 + i;
        float v = acc[q][m][i];
        if (onehot) v = v + onehot[act[row] * MZH_F + col];
        v = v + bias;
        if (jobs[q].relu) v = v > 0.0f ? v : 0.0f;
        jobs[q].out[row * jobs[q].ldo + mzh_kpos(col)] = v;  // outputs feed the next layer's A
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Pipelined chunks: a chunk is NJ output tiles (16 columns each) sharing one A operand,
// K = 16*KB with NJ*KB <= 16, so a chunk's B fragments are exactly 16 float4 per lane.  Each wave
// fetches the NEXT chunk's weights (and biases) while its MFMAs consume the current one; loads stay
// in flight across __syncthreads (no LDS-DMA is outstanding, so the barrier does not drain them).
// ------------------------------------------------------------------------------------------
// the MLP's phase barrier (a functor, so a kernel can supply a sub-group barrier)
struct MzhSyncBar {
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

// Weight chunks address the packed blob through one buffer resource: a tile is a uniform byte
// offset (one SGPR instead of a 64-bit pointer), the lane's slot a VGPR offset, so no load costs
// VALU address arithmetic.
struct MzhChunk {
  const float* wbase;  // the packed weight blob
  int woff[4];         // byte offset of each tile's fragments
  int boff[4];         // byte offset of each tile's first bias
  float* out[4];       // LDS output base per tile (a chunk may span two layers sharing A)
  int col0[4];
  int ldo, nj;         // nj: active tiles (wave-uniform), <= NJ
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mzh_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ floatx4 mzh_ld4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ float mzh_ld1(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

__device__ __forceinline__ MzhChunk mzh_chunk(const MzhNet& net, const MzhLayer& L, int nt0, int nj, float* out,
                                              int ldo) {
  MzhChunk c;
  c.ldo = ldo;
  c.nj = nj;
  c.wbase = net.wbase;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int nt = nt0 + (q < nj ? q : 0);
    c.woff[q] = L.woff + nt * L.kb * 1024;
    c.boff[q] = L.boff + nt * 64;
    c.col0[q] = nt * 16;
    c.out[q] = out;
  }
  return c;
}

// loads issued in consumption order (k-block major, the tiles of a k-block together), biases last:
// the MFMAs of k-block 0 wait only for the oldest NJ fragments, not for the whole chunk
template <int NJ, int KB, bool ALL = false>
__device__ __forceinline__ void mzh_fetch(floatx4* f, float* bv, const MzhChunk& c, int lane) {
  static_assert(NJ * KB <= 16, "chunk too large");
  const __amdgpu_buffer_rsrc_t rs = mzh_rsrc(c.wbase);
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
    for (int q = 0; q < NJ; ++q) {
      if (ALL || q < c.nj) f[q * KB + kb] = mzh_ld4(rs, 16 * lane, c.woff[q] + kb * 1024);
    }
  }
#pragma unroll
  for (int q = 0; q < NJ; ++q)
    if (ALL || q < c.nj) bv[q] = mzh_ld1(rs, 4 * (lane & 15), c.boff[q]);
}

// acc = A[rows][0:16KB] . W-tiles ; epilogue (+onehot) + bias (+relu) -> LDS
// ALL: every tile of the chunk is active (compile-time: no per-tile branches).
// NAT: the output is a logit buffer -- natural column order, padding columns past the row stride
// dropped; otherwise the output feeds a later layer's A operand and is stored in k-block order.
// oht / act (dynamics layer 1): + the one-hot action column oht[act[row] * 256 + col] (k = 64 + a),
// gathered after the first k-block's A reads so the chain does not wait for it.
// PT > 0: ring refill -- the fragments of the chunk `pc` (PT of them, contiguous from pc->w[0] in
// slot order) are loaded into f as this chain frees its slots (slot q*KB + kb after k-block kb;
// slots this chunk does not use at once), and its PNB biases into bv after the epilogue.  The
// loads of the chunk after next are spread over this chain's MFMAs instead of issuing as one burst
// that stalls every wave on the CU's address unit.
// The last k-block runs tile-major, each tile's epilogue right behind its last MFMA, so the
// stores of tile q overlap the MFMAs of tiles q+1.. instead of trailing the chain.
struct MzhNoMid {
  __device__ __forceinline__ void operator()(int) const {}
};
// MID (optional): independent VALU / LDS work, mid(kb) placed in the region of k-block kb's MFMAs, so
// it issues under their execution instead of on the phase's critical path (the latent normalisation
// beside rwd0; it must neither read this chain's output nor write its A operand or its LDS output)
// K-split chains (8-fragment chunks, mzh_mlp_recurrent_c8): KOFF = the chunk's first k-block of the
// layer (its A operand is read from there on); ACCIN: the chain continues from accio (the previous
// chunk's partial accumulators -- the same k-ordered fp32 FMA chain, only split across two calls);
// EPI = false: no epilogue, the partial accumulators are left in accio.
template <int MT, int NJ, int KB, bool ALL = false, int PT = 0, int PNB = 0, bool NAT = false, class MID = MzhNoMid,
          int KOFF = 0, bool ACCIN = false, bool EPI = true>
__device__ __forceinline__ void mzh_mma_store(floatx4* f, float* bv, const MzhChunk& c, const float* A, int lda,
                                              bool relu, const float* oht, const int* act, int lane,
                                              const MzhChunk* pc = nullptr, const floatx4* areg = nullptr,
                                              MID mid = MID{}, floatx4* accio = nullptr) {
  // areg (optional): the A operand of all KB k-blocks already in registers, [kb * MT + m] (chunks
  // of one phase that share A load it once)
  static_assert(PT <= 16 && PNB <= 4, "ring chunk too large");
  const int r = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t prs = mzh_rsrc(PT > 0 ? pc->wbase : c.wbase);
  const int pw = PT > 0 ? pc->woff[0] : 0;
  auto refill = [&](int slot) { f[slot] = mzh_ld4(prs, 16 * lane, pw + slot * 1024); };
  auto fs = [](int q, int kb) { return q * KB + kb; };
#pragma unroll
  for (int slot = NJ * KB; slot < PT; ++slot) refill(slot);
  floatx4 acc[NJ][MT];
#pragma unroll
  for (int q = 0; q < NJ; ++q)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[q][m] = ACCIN ? accio[q * MT + m] : floatx4{0.f, 0.f, 0.f, 0.f};
  // A operands double-buffered one k-block ahead: block kb + 1's LDS reads are issued before block
  // kb's MFMAs (pinned by the scheduling barrier), so a K = 256 chain does not wait on LDS latency
  // between its MFMAs
  floatx4 a[2][MT];  // [buffer][row tile]: k-steps j = 0..3 of one k-block (A in k-block order)
  const float* arow = A + r * lda + 4 * g + 16 * KOFF;
  if (!areg) {
#pragma unroll
    for (int m = 0; m < MT; ++m) a[0][m] = *reinterpret_cast<const floatx4*>(arow + m * 16 * lda);
  }
  auto aop = [&](int kb, int m) -> const floatx4& { return areg ? areg[kb * MT + m] : a[kb & 1][m]; };
  // the one-hot columns: the row actions are read here, the column values (only the epilogue adds
  // them) in k-block 1's region, under the MFMAs of k-block 0
  float oh[NJ * MT * 4];
  int acts[MT * 4];
  if (oht) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) acts[m * 4 + i] = act[m * 16 + g * 4 + i];
  }
  // LDS addresses as one lane base per row (gather) or per tile (epilogue) plus compile-time element
  // offsets, so every ds_read / ds_write takes its offset as an immediate: an index added before the
  // byte scaling cost two VALU per element (v_add_u32 + v_lshl_add_u32) -- ~290 a wave and simulation
  // at 32 roots, each an issue slot of the MFMA stream.  The one-hot chunk's tiles are consecutive
  // (mzh_chunk: col0[q] = col0[0] + 16q).
  auto gather_oh = [&]() {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float* ohrow = oht + acts[m * 4 + i] * MZH_F + (c.col0[0] + r);
#pragma unroll
        for (int q = 0; q < NJ; ++q) oh[(q * MT + m) * 4 + i] = ohrow[16 * q];
      }
  };
  auto epilogue = [&](int q) {
    // output column col0 + r; a hidden / latent unit is stored at its k-block-order position
    const int pos = c.col0[q] + (NAT ? r : 4 * (r & 3) + (r >> 2));
    if ((ALL || q < c.nj) && (!NAT || pos < c.ldo)) {
      float* ob = c.out[q] + (g * 4 * c.ldo + pos);  // row g * 4 of row tile 0
#pragma unroll
      for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[q][m][i];
          if (oht) v = v + oh[(q * MT + m) * 4 + i];
          v = v + bv[q];
          if (relu) v = v > 0.0f ? v : 0.0f;
          ob[(m * 16 + i) * c.ldo] = v;
        }
      }
    }
  };
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 1 < KB && !areg) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        a[(kb + 1) & 1][m] = *reinterpret_cast<const floatx4*>(arow + m * 16 * lda + (kb + 1) * 16);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (oht && kb == (KB > 1 ? 1 : 0)) gather_oh();
    mid(kb);
    if (kb + 1 < KB) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int q = 0; q < NJ; ++q) {
          if (ALL || q < c.nj) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[q][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(aop(kb, m)[j], f[fs(q, kb)][j], acc[q][m], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < NJ; ++q)
        if (fs(q, kb) < PT) refill(fs(q, kb));
    } else {  // last k-block: tile-major, epilogue behind each tile
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
        if (ALL || q < c.nj) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[q][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(aop(kb, m)[j], f[fs(q, kb)][j], acc[q][m], 0, 0, 0);
        }
        if (fs(q, kb) < PT) refill(fs(q, kb));
        if (EPI) epilogue(q);
      }
    }
  }
  if (!EPI) {
#pragma unroll
    for (int q = 0; q < NJ; ++q)
#pragma unroll
      for (int m = 0; m < MT; ++m) accio[q * MT + m] = acc[q][m];
  }
#pragma unroll
  for (int q = 0; q < PNB; ++q) bv[q] = mzh_ld1(prs, 4 * (lane & 15), pc->boff[q]);
}

// normalize_h_state (networks.py:191-196): 8 lanes per row, 8 elements per lane.
// a / b for a >= 0 and a normal b > 0, from y = RN(1/b) (Markstein: q = RN(a*y), the fma residual
// is exact, one correction step gives RN(a/b)).  Exact unless the residual can underflow: `slow`
// flags a != 0 with a or the quotient below 2^-100, and the caller redoes the wave with IEEE
// division (tests/test_markstein.py checks the fp32 and fp64 forms against true division).
__device__ __forceinline__ float mzh_fdiv(float a, float b, float y, bool& slow) {
  const float q = a * y;
  const float r = __builtin_fmaf(-q, b, a);
  const float res = __builtin_fmaf(r, y, q);
  slow |= (a != 0.0f) & ((a < 0x1p-100f) | (res < 0x1p-100f));
  return res;
}

// One pass over the rows in three steps -- load (LDS read), reduce (row min / max), finish (the
// quotients, LDS store) -- so a caller can spread it over an MFMA chain.  finish<false>: the Markstein
// quotients; returns whether some lane of the wave flagged `slow` (wave-uniform), in which case the
// caller reruns the pass with finish<true> (IEEE division, the same results wherever the Markstein
// form is exact).  src is left untouched, so the rerun may come later.
//   R == 16: 16 rows over all 256 threads -- 16 lanes per row (one DPP row), 4 elements per lane, so
//   all four waves share the work (8 lanes per row leave waves 2, 3 idle at the next barrier); with
//   the dynamics one-hot columns in LDS for 16-root tiles too: 4,096 roots 0.921 -> 0.910 ms.
//   Otherwise 8 lanes per row, 8 elements per lane, R / 32 rows per thread.
template <int R>
struct MzhNormPass {
  static constexpr int NE = R == 16 ? 4 : 8, NR = R == 16 ? 1 : R / 32;
  static_assert(R == 16 || R % 32 == 0, "normalisation rows");
  float v[NR][NE];
  float mn[NR];
  __device__ __forceinline__ int off(int tid, int k) const {
    return R == 16 ? (tid >> 4) * MZH_LD64 + (tid & 15) * 4 : (k * 32 + (tid >> 3)) * MZH_LD64 + (tid & 7) * 8;
  }
  __device__ __forceinline__ void load(const float* src, int tid) {
#pragma unroll
    for (int k = 0; k < NR; ++k)
#pragma unroll
      for (int h = 0; h < NE; h += 4) {
        const floatx4 t = *reinterpret_cast<const floatx4*>(src + off(tid, k) + h);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[k][h + i] = t[i];
      }
  }
  float d[NR];
  __device__ __forceinline__ void reduce() {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      float lo = v[k][0], hi = v[k][0];
#pragma unroll
      for (int i = 1; i < NE; ++i) {
        lo = mzh_vmin(v[k][i], lo);
        hi = mzh_vmax(v[k][i], hi);
      }
      lo = mzh_min8_nonan(lo);
      hi = mzh_max8_nonan(hi);
      if (R == 16) {  // the two 8-lane halves of the row (row_ror:8)
        const float tn = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(lo), 0x128, 0xF, 0xF, true));
        const float tx = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(hi), 0x128, 0xF, 0xF, true));
        lo = mzh_vmin(tn, lo);
        hi = mzh_vmax(tx, hi);
      }
      mn[k] = lo;
      d[k] = (hi - lo) + 9.999999939225290290778502821922302246094e-09f;
    }
  }
  template <bool EXACT>
  __device__ __forceinline__ bool finish(float* dst, int tid) const {
    bool slow = false;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      float o[NE];
      if (EXACT) {
#pragma unroll
        for (int i = 0; i < NE; ++i) o[i] = (v[k][i] - mn[k]) / d[k];
      } else {
        const float y = 1.0f / d[k];
#pragma unroll
        for (int i = 0; i < NE; ++i) o[i] = mzh_fdiv(v[k][i] - mn[k], d[k], y, slow);
      }
#pragma unroll
      for (int h = 0; h < NE; h += 4)
        *reinterpret_cast<floatx4*>(dst + off(tid, k) + h) = floatx4{o[h], o[h + 1], o[h + 2], o[h + 3]};
    }
    return !EXACT && __ballot(slow) != 0;
  }
};

template <int R, bool EXACT>
__device__ __forceinline__ bool mzh_normalize_rows(const float* src, float* dst, int tid) {
  MzhNormPass<R> n;
  n.load(src, tid);
  n.reduce();
  return n.template finish<EXACT>(dst, tid);
}

template <int R>
__device__ __forceinline__ void mzh_normalize_par(const float* src, float* dst, int tid) {
  if (__builtin_expect(mzh_normalize_rows<R, false>(src, dst, tid), 0)) mzh_normalize_rows<R, true>(src, dst, tid);
}

// Heads (networks.py:83,109,152-189): 8 lanes per row; the value and reward heads of a row run
// interleaved on the same lanes (independent chains), the policy softmax alongside.  Lane q owns
// logits k = q + 8i; max / exp / divide are lane-parallel, and both 33-term sums use the fixed
// order of sum8_tree in the oracle: sequential per-lane partials combined by the DPP tree.
// SUP: the support size when the caller knows it at compile time (0: runtime `support`).  Logit
// loads are unconditional (every k < 40 lies inside the row stride) and masked by selects, so
// the head runs branch-free.
// The row's results also come back in registers (MzhHeadOut: lane q's policy probability; value and
// reward on lane 0); STORE = false skips the LDS copies (the search kernel keeps them in registers).
struct MzhHeadOut {
  float pp, value, reward;
};
// CHAIN32 = false: bin 32 of a 33-bin head is already in lval / lrwd (mzh_bin32_wave ran in the MLP).
template <int R, int SUP = 0, bool STORE = true, bool CHAIN32 = true, class SM>
__device__ __forceinline__ MzhHeadOut mzh_heads_row(SM& sm, const MzhNet& net, int row, int q, int support_in,
                                                   bool recurrent) {
  const int support = SUP ? SUP : support_in;
  // bin 32 of the reward (lanes 0-3) and value (lanes 4-7) logits: lane c of the quad runs chain c over
  // hidden units 16b + 4j + c -- LDS positions 16b + 4c + j (k-block order), one ds_read_b128 per block
  float l32r = 0.0f, l32v = 0.0f;
  if (CHAIN32 && support == 33) {
    const int hv = q >> 2, c = q & 3;
    const float* hid = (hv ? sm.hidV : sm.hidR) + row * MZH_LD256 + 4 * c;
    const float4* w = (hv ? net.val32 : net.rwd32) + c;
    float acc = 0.0f;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const floatx4 a4 = *reinterpret_cast<const floatx4*>(hid + 16 * b);
      const float4 w4 = w[4 * b];
      acc = __builtin_fmaf(a4[0], w4.x, acc);
      acc = __builtin_fmaf(a4[1], w4.y, acc);
      acc = __builtin_fmaf(a4[2], w4.z, acc);
      acc = __builtin_fmaf(a4[3], w4.w, acc);
    }
    acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0xB1, 0xF, 0xF, true));  // p0+p1 | p2+p3
    acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x4E, 0xF, 0xF, true));  // (p0+p1)+(p2+p3)
    const float l32 = acc + (hv ? net.val32b : net.rwd32b);
    l32r = l32;  // valid on lanes 0-3
    l32v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(l32), 0x104, 0xF, 0xF, true));  // row_shl:4: lane 4 -> 0
    if (STORE) {
      if (q == 4) sm.lval[row * MZH_LDSUP + 32] = l32;
      if (q == 0 && recurrent) sm.lrwd[row * MZH_LDSUP + 32] = l32;
    }
  }
  const float lraw = sm.lpol[row * MZH_LDPOL + q];
  const float lg = q < MZH_A ? lraw : -__builtin_inff();
  MzhHeadOut out{0.0f, 0.0f, 0.0f};
  if (support == 1) {
    out.value = sm.lval[row * MZH_LDSUP];
    out.reward = recurrent ? sm.lrwd[row * MZH_LDSUP] : 0.0f;
    if (STORE && q == 0) {
      sm.value[row] = out.value;
      sm.reward[row] = out.reward;
    }
  }
  const int nh = support == 1 ? 0 : (recurrent ? 2 : 1);
  const float* lv[2] = {sm.lval + row * MZH_LDSUP, sm.lrwd + row * MZH_LDSUP};
  float e[2][5], m[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    m[h] = -__builtin_inff();
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = q + 8 * i;
      // bin 32 (lane 0, i = 4) from the vector chains above
      const float raw = (CHAIN32 && i == 4) ? (h ? l32r : l32v) : lv[h][k];
      e[h][i] = (h < nh && k < 33) ? raw : -__builtin_inff();
      m[h] = __builtin_fmaxf(e[h][i], m[h]);  // NaN-free; the max only feeds exponent arguments
    }
  }
  const float mp = mzh_max8_nonan(lg);
#pragma unroll
  for (int h = 0; h < 2; ++h) m[h] = mzh_max8_nonan(m[h]);
  // every exponent argument is <= 0; xmin tracks the smallest one that feeds a probability
  const float xp = lg - mp;
  const float epx = mzh_expf_np(xp);  // every lane (no divergent branch); lanes 6, 7 discard it
  const float ep = q < MZH_A ? epx : 0.0f;
  float xmin = q < MZH_A ? xp : 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const float xv = e[h][i] - m[h];
      const float ex = mzh_expf_np(xv);  // every lane (no divergent branch)
      e[h][i] = (q + 8 * i < 33) ? ex : 0.0f;
      if (h < nh && q + 8 * i < 33) xmin = __builtin_fminf(xv, xmin);
    }
  float sh[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float a = e[h][0];
#pragma unroll
    for (int i = 1; i < 4; ++i) a = a + e[h][i];
    if (q == 0) a = a + e[h][4];
    sh[h] = a;
  }
  const float sp = mzh_sum8(ep);
#pragma unroll
  for (int h = 0; h < 2; ++h) sh[h] = mzh_sum8(sh[h]);
  // probabilities: Markstein division from one reciprocal per head, IEEE fallback when flagged.
  // The sums lie in [1, 33], so with every argument >= -65 each numerator is 0 or >= e^-65 and each
  // quotient >= e^-65 / 33 > 2^-100: the residual stays normal and the quotient is RN(a / s) (the
  // condition mzh_fdiv checks per division, decided here once per lane from the arguments)
  const bool slow = xmin < -65.0f;
  float pk[2][5];
  const float yp = 1.0f / sp;
  auto mdiv = [](float a, float b, float y) {
    const float qq = a * y;
    const float rr = __builtin_fmaf(-qq, b, a);
    return __builtin_fmaf(rr, y, qq);
  };
  float pp = mdiv(ep, sp, yp);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float y = 1.0f / sh[h];
#pragma unroll
    for (int i = 0; i < 5; ++i) pk[h][i] = mdiv(e[h][i], sh[h], y);
  }
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    pp = ep / sp;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 5; ++i) pk[h][i] = e[h][i] / sh[h];
  }
  out.pp = q < MZH_A ? pp : 0.0f;
  if (STORE && q < MZH_A) sm.pi[row * 8 + q] = pp;
  float x[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    x[h] = 0.0f;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = q + 8 * i;
      if (k < 33) {
        const float prod = pk[h][i] * (float)(k - 16);
        x[h] = i == 0 ? prod : x[h] + prod;
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) x[h] = mzh_sum8(x[h]);
  if (nh > 0) {
    const mzh_f2 vr = mzh_signed_parabolic2(mzh_f2{x[0], x[1]});  // value and reward side by side
    out.value = vr.x;
    out.reward = nh > 1 ? vr.y : 0.0f;
    if (STORE && q == 0) {
      sm.value[row] = out.value;
      sm.reward[row] = out.reward;
    }
  }
  return out;
}

// all rows: 8 lanes per row, row = tid / 8 (32 rows over 256 threads)
template <int R, bool CHAIN32 = true, class SM>
__device__ __forceinline__ void mzh_heads_par(SM& sm, const MzhNet& net, bool recurrent, int tid) {
  const int row = tid >> 3, q = tid & 7;
  if (row < R) mzh_heads_row<R, 0, true, CHAIN32>(sm, net, row, q, net.support, recurrent);
}

// LDS copy of the bin-32 weight rows (rwd32, val32) for mzh_bin32_wave; before a barrier
template <int R, class SM>
__device__ __forceinline__ void mzh_w32_fill(SM& sm, const MzhNet& net, int tid) {
  if (tid < 128) reinterpret_cast<float4*>(sm.w32)[tid] = tid < 64 ? net.rwd32[tid] : net.val32[tid - 64];
}

// Bin 32 of the 33-bin reward and value logits of all R rows on ONE wave -- the wave without a
// pol2 / val2 tile in the last MLP phase, whose slot is otherwise idle.  Chain c of oracle
// linear_head runs over hidden units 16b + 4j + c, at LDS positions 16b + 4c + j; the result is
// ((p0 + p1) + (p2 + p3)) + bias, stored to column 32 of lrwd / lval (the heads then read it like
// bins 0-31).  R = 32: lane -> (row, head), four chains per lane.  R = 16: lane -> (row, head,
// chain pair), the pairs' sums exchanged across the half-waves.  Weights come from the LDS copy
// (two distinct addresses per read: a broadcast).
template <int R, class SM>
__device__ __forceinline__ void mzh_bin32_wave(SM& sm, const MzhNet& net, int lane) {
  static_assert(R == 16 || R == 32, "rows per workgroup");
  constexpr int CH = R == 32 ? 4 : 2;  // chains per lane
  const int row = lane & (R - 1);
  const bool hv = (lane / R) & 1;  // value head / reward head
  const int c0 = R == 32 ? 0 : 2 * (lane >> 5);
  const float* hid = (hv ? sm.hidV : sm.hidR) + row * MZH_LD256 + 4 * c0;
  const floatx4* w = reinterpret_cast<const floatx4*>(sm.w32 + (hv ? 256 : 0)) + c0;
  float acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = 0.0f;
#pragma unroll
  for (int b = 0; b < 16; ++b)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const floatx4 a4 = *reinterpret_cast<const floatx4*>(hid + 16 * b + 4 * c);
      const floatx4 w4 = w[4 * b + c];
      acc[c] = __builtin_fmaf(a4[0], w4[0], acc[c]);
      acc[c] = __builtin_fmaf(a4[1], w4[1], acc[c]);
      acc[c] = __builtin_fmaf(a4[2], w4[2], acc[c]);
      acc[c] = __builtin_fmaf(a4[3], w4[3], acc[c]);
    }
  const float p = acc[0] + acc[1];
  float l32;
  if constexpr (R == 32)
    l32 = p + (acc[2] + acc[3]);
  else
    l32 = p + __shfl_xor(p, 32);
  l32 = l32 + (hv ? net.val32b : net.rwd32b);
  if (R == 32 || lane < 32) (hv ? sm.lval : sm.lrwd)[row * MZH_LDSUP + 32] = l32;
}

// The per-wave chunk schedule of the prediction function (networks.py:140-150) on sm.x:
//   C5/C6: pol0 (waves 0,1) or val0 (waves 2,3), 4 tiles each;  C7: pol2 (wave 0) / val2 (waves 1..)
template <int R, class SM>
__device__ __forceinline__ MzhChunk mzh_pred_chunk(SM& sm, const MzhNet& net, int wave, int c) {
  const int id0 = wave * 8 + c * 4;
  return id0 >= 16 ? mzh_chunk(net, net.val0, id0 - 16, 4, sm.hidV, MZH_LD256)
                   : mzh_chunk(net, net.pol0, id0, 4, sm.hidP, MZH_LD256);
}
template <int R, class SM>
__device__ __forceinline__ MzhChunk mzh_head_chunk(SM& sm, const MzhNet& net, int wave) {
  if (wave == 0) return mzh_chunk(net, net.pol2, 0, 1, sm.lpol, MZH_LDPOL);
  return mzh_chunk(net, net.val2, wave - 1 < net.val2.nt ? wave - 1 : 0, wave - 1 < net.val2.nt ? 1 : 0, sm.lval, MZH_LDSUP);
}
// waves with a pol2 / val2 tile: 0-2 for 33-bin heads (N2 = 2; wave 3 runs bin 32 by vector chains),
// 0-1 for scalar heads
template <int N2>
__device__ __forceinline__ bool mzh_has_head_tile(int wave) { return wave <= N2; }

// nj consecutive tiles of the prediction hidden layers' 32-tile strip (tiles 0-15: pol0 -> hidP,
// 16-31: val0 -> hidV; both read the normalised latent), starting at strip tile t0
template <int R, class SM>
__device__ __forceinline__ MzhChunk mzh_pred_tiles(SM& sm, const MzhNet& net, int t0, int nj) {
  MzhChunk c;
  c.ldo = MZH_LD256;
  c.nj = nj;
  c.wbase = net.wbase;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int t = t0 + (q < nj ? q : 0);
    const bool v = t >= 16;
    const MzhLayer& L = v ? net.val0 : net.pol0;
    const int nt = t & 15;
    c.woff[q] = L.woff + nt * L.kb * 1024;
    c.boff[q] = L.boff + nt * 64;
    c.col0[q] = nt * 16;
    c.out[q] = v ? sm.hidV : sm.hidP;
  }
  return c;
}

// initial_inference (networks.py:71-94): sm.x holds obs rows zero-padded to 16*rep0.kb
template <int R, class SM, class BAR = MzhSyncBar>
__device__ void mzh_mlp_initial(SM& sm, const MzhNet& net, int wave_in, int lane, BAR bar = BAR{}) {
  constexpr int MT = R / 16;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(wave_in);
  floatx4 fa[16], fb[16];
  float ba[4], bb[4];
  {  // rep0: 16 tiles, 4 per wave (K = 3N padded: runtime k-blocks)
    MzhJob jobs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) jobs[q] = mzh_job(sm.x, MZH_LD64, net.rep0, wave * 4 + q, sm.hidP, MZH_LD256, 1);
    mzh_run_jobs<MT, 4>(jobs, net.rep0.kb, nullptr, nullptr, lane);
  }
  bar();
  {  // rep2: 4 tiles, 1 per wave
    MzhJob job = mzh_job(sm.hidP, MZH_LD256, net.rep2, wave, sm.hraw, MZH_LD64, 0);
    mzh_run_jobs<MT, 1>(&job, net.rep2.kb, nullptr, nullptr, lane);
  }
  const MzhChunk c5 = mzh_pred_chunk<R>(sm, net, wave, 0), c6 = mzh_pred_chunk<R>(sm, net, wave, 1);
  const MzhChunk c7 = mzh_head_chunk<R>(sm, net, wave);
  mzh_fetch<4, 4, true>(fa, ba, c5, lane);
  mzh_fetch<4, 4, true>(fb, bb, c6, lane);
  bar();
  mzh_normalize_par<R>(sm.hraw, sm.x, tid);
  bar();
  mzh_mma_store<MT, 4, 4, true>(fa, ba, c5, sm.x, MZH_LD64, true, nullptr, nullptr, lane);
  mzh_fetch<1, 16>(fa, ba, c7, lane);
  mzh_mma_store<MT, 4, 4, true>(fb, bb, c6, sm.x, MZH_LD64, true, nullptr, nullptr, lane);
  bar();
  mzh_mma_store<MT, 1, 16, false, 0, 0, true>(fa, ba, c7, c7.out[0] == sm.lpol ? sm.hidP : sm.hidV, MZH_LD256, false,
                                            nullptr, nullptr, lane);
  bar();
  mzh_heads_par<R>(sm, net, false, tid);
  bar();
}

// recurrent_inference (networks.py:96-138), split so the first two chunks' weights (dyn0, dyn2)
// can be fetched early -- across the search kernel's tree phase -- into fa/fb:
//   mzh_mlp_fetch12 : issue the loads of chunk 1 (dyn0) into fa and chunk 2 (dyn2) into fb
//   mzh_mlp_recurrent_body<R, NEXT> : the MLP; with NEXT it re-issues fetch12 for the next step
// Input: sm.x = parent latents, sm.act = actions.  Output: sm.x = normalised new latent,
// sm.pi / sm.value / sm.reward.
template <int R, class SM>
__device__ __forceinline__ void mzh_mlp_fetch12(SM& sm, const MzhNet& net, int wave_in, int lane, floatx4* fa,
                                                float* ba, floatx4* fb, float* bb) {
  const int wave = __builtin_amdgcn_readfirstlane(wave_in);
  mzh_fetch<4, 4, true>(fa, ba, mzh_chunk(net, net.dyn0, wave * 4, 4, sm.hidP, MZH_LD256), lane);
  mzh_fetch<1, 16, true>(fb, bb, mzh_chunk(net, net.dyn2, wave, 1, sm.hraw, MZH_LD64), lane);
}

// N2 = reward / value layer-2 tiles (2: 33-bin support, bins 0-31; 1: scalar); HEADS: finish with the heads on
// all rows (standalone inference) -- the search kernel runs each root's heads itself.
template <int R, bool NEXT, int N2, bool HEADS, class SM, class BAR = MzhSyncBar>
__device__ __forceinline__ void mzh_mlp_recurrent_body(SM& sm, const MzhNet& net, int wave_in, int lane,
                                                       floatx4* fa, float* ba, floatx4* fb, float* bb,
                                                       const float* onehot, BAR bar = BAR{}) {
  constexpr int MT = R / 16;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(wave_in);  // wave-uniform -> chunk descriptors in SGPRs
  // Weight chunks alternate between the two fragment buffers, each refilled by the chain that
  // consumes it (ring, mzh_mma_store PT) with the chunk two steps ahead:
  //   fa: dyn0 -> rwd0 -> P2 -> pol2/val2 -> next dyn0      fb: dyn2 -> rwd2 | P1 -> P3 -> next dyn2
  // Phase B (after rwd0) balances rwd2 against the prediction hidden layers: waves w < N2 run one
  // rwd2 tile (K = 256, 4 units) + N2 + 4 prediction tiles (K = 64, 1 unit each), the others N2 + 8
  // prediction tiles -- 8 + N2 units per wave.
  const bool r2 = wave < N2;
  const int P1 = r2 ? wave * (N2 + 4) : N2 * (N2 + 4) + (wave - N2) * (N2 + 8);
  const int P2 = P1 + (r2 ? 0 : 4), P3 = P2 + 4;
  const bool ht = mzh_has_head_tile<N2>(wave);
  const MzhChunk c_rwd0 = mzh_chunk(net, net.rwd0, wave * 4, 4, sm.hidR, MZH_LD256);
  const MzhChunk c_p2 = mzh_pred_tiles<R>(sm, net, P2, 4);
  MZH_STAMP_DECL
  MZH_STAMP(0);
  mzh_mma_store<MT, 4, 4, true, 16, 4>(fa, ba, mzh_chunk(net, net.dyn0, wave * 4, 4, sm.hidP, MZH_LD256), sm.x, MZH_LD64,
                                       true, onehot, sm.act, lane, &c_rwd0);  // dyn0 + one-hot + bias, relu
  MZH_STAMP(1);
  bar();
  MZH_STAMP(2);
  {
    const MzhChunk c_b = r2 ? mzh_chunk(net, net.rwd2, wave, 1, sm.lrwd, MZH_LDSUP) : mzh_pred_tiles<R>(sm, net, P1, 4);
    mzh_mma_store<MT, 1, 16, true, 16, 4>(fb, bb, mzh_chunk(net, net.dyn2, wave, 1, sm.hraw, MZH_LD64), sm.hidP, MZH_LD256,
                                          false, nullptr, nullptr, lane, &c_b);  // dyn2 -> h'
  }
  MZH_STAMP(3);
  bar();
  MZH_STAMP(4);
  MZH_STAMP(5);
  // rwd0 on h' (networks.py:132); the normalisation only reads h' too (writing sm.x, read after the
  // next barrier): its pass issues under rwd0's MFMAs, the rare exact rerun after them
  MzhNormPass<R> norm;
  bool slow = false;
  mzh_mma_store<MT, 4, 4, true, 16, 4>(fa, ba, c_rwd0, sm.hraw, MZH_LD64, true, nullptr, nullptr, lane, &c_p2,
                                       nullptr, [&](int kb) {
                                         if (kb == 0) norm.load(sm.hraw, tid);
                                         if (kb == 1) norm.reduce();
                                         if (kb == 2) slow = norm.template finish<false>(sm.x, tid);
                                       });
  if (__builtin_expect(slow, 0)) norm.template finish<true>(sm.x, tid);
  MZH_STAMP(6);
  bar();
  MZH_STAMP(7);
  {
    // the prediction chunks of this phase (P1, P2, P3) all read the normalised latent sm.x: its four
    // k-blocks are loaded into registers once
    floatx4 ax[4 * MT];
    {
      const float* arow = sm.x + (lane & 15) * MZH_LD64 + 4 * (lane >> 4);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int m = 0; m < MT; ++m) ax[kb * MT + m] = *reinterpret_cast<const floatx4*>(arow + m * 16 * MZH_LD64 + kb * 16);
    }
    const MzhChunk c_p3 = mzh_pred_tiles<R>(sm, net, P3, N2);
    if (r2)
      mzh_mma_store<MT, 1, 16, true, 4 * N2, N2, true>(fb, bb, mzh_chunk(net, net.rwd2, wave, 1, sm.lrwd, MZH_LDSUP),
                                                       sm.hidR, MZH_LD256, false, nullptr, nullptr, lane,
                                                       &c_p3);  // rwd2 -> reward logits
    else
      mzh_mma_store<MT, 4, 4, true, 4 * N2, N2>(fb, bb, mzh_pred_tiles<R>(sm, net, P1, 4), sm.x, MZH_LD64, true,
                                                nullptr, nullptr, lane, &c_p3, ax);
    MZH_STAMP(8);
    if (ht) {
      const MzhChunk c_h = mzh_head_chunk<R>(sm, net, wave);
      mzh_mma_store<MT, 4, 4, true, 16, 1>(fa, ba, c_p2, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &c_h, ax);
    } else {
      mzh_mma_store<MT, 4, 4, true>(fa, ba, c_p2, sm.x, MZH_LD64, true, nullptr, nullptr, lane, nullptr, ax);
    }
    if (NEXT) {
      const MzhChunk c_n2 = mzh_chunk(net, net.dyn2, wave, 1, sm.hraw, MZH_LD64);
      mzh_mma_store<MT, N2, 4, true, 16, 1>(fb, bb, c_p3, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &c_n2, ax);
    } else {
      mzh_mma_store<MT, N2, 4, true>(fb, bb, c_p3, sm.x, MZH_LD64, true, nullptr, nullptr, lane, nullptr, ax);
    }
  }
  MZH_STAMP(9);
  bar();
  {
    const MzhChunk c_n1 = mzh_chunk(net, net.dyn0, wave * 4, 4, sm.hidP, MZH_LD256);
    if (ht) {
      const MzhChunk c_h = mzh_head_chunk<R>(sm, net, wave);
      float* hin = wave == 0 ? sm.hidP : sm.hidV;
      if (NEXT)
        mzh_mma_store<MT, 1, 16, true, 16, 4, true>(fa, ba, c_h, hin, MZH_LD256, false, nullptr, nullptr, lane,
                                                    &c_n1);  // pol2 / val2
      else
        mzh_mma_store<MT, 1, 16, true, 0, 0, true>(fa, ba, c_h, hin, MZH_LD256, false, nullptr, nullptr, lane);
    } else {
      if (NEXT) mzh_fetch<4, 4, true>(fa, ba, c_n1, lane);  // next step's dyn0 chunk
      if (N2 == 2) mzh_bin32_wave<R>(sm, net, lane);      // 33-bin heads: wave 3 (no head tile) runs bin 32
    }
  }
  MZH_STAMP(10);
  bar();
  if (HEADS) {
    mzh_heads_par<R, N2 != 2>(sm, net, true, tid);
    MZH_STAMP(11);
    bar();
  }
  MZH_STAMP(12);
}

// ------------------------------------------------------------------------------------------
// The same recurrent MLP for a 16-root tile whose workgroup shares its CU with a second one (the
// two-workgroups-per-CU cooperative kernel, mzh_search_occ2_kernel): <= 256 registers a lane, so the
// weight ring is two buffers of 8 fragments (fa8, fb8) instead of 16, and every 16-fragment chunk
// of mzh_mlp_recurrent_body is two 8-fragment chunks -- K = 64 layers two tiles per chunk, K = 256
// tiles two k-halves (mzh_mma_store KOFF / ACCIN / EPI: one k-ordered chain split across two calls,
// the same FMAs in the same order).  Chunk i runs from buffer i % 2 and refills it with chunk i + 2
// as its MFMAs free the slots; per simulation
//   A1 A2 | B1 B2 | C1 C2 | D1 .. D5 | E1 E2        (E: the waves with a pol2 / val2 tile)
// so waves with a head tile run 13 chunks and the others 11: the next simulation's A1 / A2 arrive in
// the swapped buffers and the caller swaps fa8 / fb8 before the next call (mzh_c8_swap, after the
// tree phase, when those loads have long completed).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ MzhChunk mzh_chunk_khalf(MzhChunk c) {  // the second k-half of a K = 256 tile
  c.woff[0] += 8 * 1024;
  return c;
}

template <class SM>
__device__ __forceinline__ void mzh_mlp_fetch12_c8(SM& sm, const MzhNet& net, int wave_in, int lane, floatx4* fa,
                                                   float* ba, floatx4* fb, float* bb) {
  const int wave = __builtin_amdgcn_readfirstlane(wave_in);
  mzh_fetch<2, 4, true>(fa, ba, mzh_chunk(net, net.dyn0, wave * 4, 2, sm.hidP, MZH_LD256), lane);
  mzh_fetch<2, 4, true>(fb, bb, mzh_chunk(net, net.dyn0, wave * 4 + 2, 2, sm.hidP, MZH_LD256), lane);
}

__device__ __forceinline__ void mzh_c8_swap(floatx4* fa, float* ba, floatx4* fb, float* bb) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const floatx4 t = fa[i];
    fa[i] = fb[i];
    fb[i] = t;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float t = ba[i];
    ba[i] = bb[i];
    bb[i] = t;
  }
}

template <int N2, class SM>
__device__ __forceinline__ void mzh_mlp_recurrent_c8(SM& sm, const MzhNet& net, int wave_in, int lane, floatx4* fa,
                                                     float* ba, floatx4* fb, float* bb, const float* onehot) {
  constexpr int R = 16, MT = 1;
  const int tid = threadIdx.x;
  int wave = __builtin_amdgcn_readfirstlane(wave_in);
  // opaque to the optimiser: the 13 chunk descriptors below are rebuilt each simulation (a few SALU)
  // instead of being hoisted out of the simulation loop, where they would stay live in SGPRs across the
  // tree phase and spill
  asm volatile("" : "+s"(wave));
  const bool r2 = wave < N2;
  const int P1 = r2 ? wave * (N2 + 4) : N2 * (N2 + 4) + (wave - N2) * (N2 + 8);
  const int P2 = P1 + (r2 ? 0 : 4), P3 = P2 + 4;
  const bool ht = mzh_has_head_tile<N2>(wave);
  const MzhChunk cA1 = mzh_chunk(net, net.dyn0, wave * 4, 2, sm.hidP, MZH_LD256);
  const MzhChunk cA2 = mzh_chunk(net, net.dyn0, wave * 4 + 2, 2, sm.hidP, MZH_LD256);
  const MzhChunk cB1 = mzh_chunk(net, net.dyn2, wave, 1, sm.hraw, MZH_LD64), cB2 = mzh_chunk_khalf(cB1);
  const MzhChunk cC1 = mzh_chunk(net, net.rwd0, wave * 4, 2, sm.hidR, MZH_LD256);
  const MzhChunk cC2 = mzh_chunk(net, net.rwd0, wave * 4 + 2, 2, sm.hidR, MZH_LD256);
  const MzhChunk cR1 = mzh_chunk(net, net.rwd2, wave, 1, sm.lrwd, MZH_LDSUP), cR2 = mzh_chunk_khalf(cR1);
  const MzhChunk cD1 = r2 ? cR1 : mzh_pred_tiles<R>(sm, net, P1, 2);
  const MzhChunk cD2 = r2 ? cR2 : mzh_pred_tiles<R>(sm, net, P1 + 2, 2);
  const MzhChunk cD3 = mzh_pred_tiles<R>(sm, net, P2, 2), cD4 = mzh_pred_tiles<R>(sm, net, P2 + 2, 2);
  const MzhChunk cD5 = mzh_pred_tiles<R>(sm, net, P3, N2);
  const MzhChunk cE1 = mzh_head_chunk<R>(sm, net, wave), cE2 = mzh_chunk_khalf(cE1);
  floatx4 acc[2];
  // ---- A: dyn0 + one-hot + bias, relu -> hidP (networks.py:129-131)
  mzh_mma_store<MT, 2, 4, true, 8, 1>(fa, ba, cA1, sm.x, MZH_LD64, true, onehot, sm.act, lane, &cB1);
  mzh_mma_store<MT, 2, 4, true, 8, 1>(fb, bb, cA2, sm.x, MZH_LD64, true, onehot, sm.act, lane, &cB2);
  __syncthreads();
  // ---- B: dyn2 -> h' (one K = 256 chain in two halves)
  mzh_mma_store<MT, 1, 8, true, 8, 2, false, MzhNoMid, 0, false, false>(fa, ba, cB1, sm.hidP, MZH_LD256, false, nullptr,
                                                                      nullptr, lane, &cC1, nullptr, MzhNoMid{}, acc);
  mzh_mma_store<MT, 1, 8, true, 8, 2, false, MzhNoMid, 8, true, true>(fb, bb, cB2, sm.hidP, MZH_LD256, false, nullptr,
                                                                     nullptr, lane, &cC2, nullptr, MzhNoMid{}, acc);
  __syncthreads();
  // ---- C: rwd0 on h' (networks.py:132), the latent normalisation under its MFMAs
  MzhNormPass<R> norm;
  bool slow = false;
  if (r2) {
    mzh_mma_store<MT, 2, 4, true, 8, 1>(fa, ba, cC1, sm.hraw, MZH_LD64, true, nullptr, nullptr, lane, &cD1, nullptr,
                                        [&](int kb) {
                                          if (kb == 0) norm.load(sm.hraw, tid);
                                          if (kb == 1) norm.reduce();
                                          if (kb == 2) slow = norm.template finish<false>(sm.x, tid);
                                        });
    mzh_mma_store<MT, 2, 4, true, 8, 1>(fb, bb, cC2, sm.hraw, MZH_LD64, true, nullptr, nullptr, lane, &cD2);
  } else {
    mzh_mma_store<MT, 2, 4, true, 8, 2>(fa, ba, cC1, sm.hraw, MZH_LD64, true, nullptr, nullptr, lane, &cD1, nullptr,
                                        [&](int kb) {
                                          if (kb == 0) norm.load(sm.hraw, tid);
                                          if (kb == 1) norm.reduce();
                                          if (kb == 2) slow = norm.template finish<false>(sm.x, tid);
                                        });
    mzh_mma_store<MT, 2, 4, true, 8, 2>(fb, bb, cC2, sm.hraw, MZH_LD64, true, nullptr, nullptr, lane, &cD2);
  }
  if (__builtin_expect(slow, 0)) norm.template finish<true>(sm.x, tid);
  __syncthreads();
  // ---- D: rwd2 (waves < N2) and the prediction hidden layers (networks.py:140-150) on sm.x
  {
    floatx4 ax[4];
    {
      const float* arow = sm.x + (lane & 15) * MZH_LD64 + 4 * (lane >> 4);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) ax[kb] = *reinterpret_cast<const floatx4*>(arow + kb * 16);
    }
    if (r2) {
      mzh_mma_store<MT, 1, 8, true, 8, 2, true, MzhNoMid, 0, false, false>(fa, ba, cD1, sm.hidR, MZH_LD256, false, nullptr,
                                                                         nullptr, lane, &cD3, nullptr, MzhNoMid{}, acc);
      mzh_mma_store<MT, 1, 8, true, 8, 2, true, MzhNoMid, 8, true, true>(fb, bb, cD2, sm.hidR, MZH_LD256, false, nullptr,
                                                                       nullptr, lane, &cD4, nullptr, MzhNoMid{}, acc);
    } else {
      mzh_mma_store<MT, 2, 4, true, 8, 2>(fa, ba, cD1, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cD3, ax);
      mzh_mma_store<MT, 2, 4, true, 8, 2>(fb, bb, cD2, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cD4, ax);
    }
    // D3 refills its buffer with D5 (N2 tiles); D4 with E1 (head waves) or the next simulation's A1
    mzh_mma_store<MT, 2, 4, true, 4 * N2, N2>(fa, ba, cD3, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cD5, ax);
    if (ht) {
      mzh_mma_store<MT, 2, 4, true, 8, 1>(fb, bb, cD4, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cE1, ax);
      mzh_mma_store<MT, N2, 4, true, 8, 1>(fa, ba, cD5, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cE2, ax);
    } else {
      mzh_mma_store<MT, 2, 4, true, 8, 2>(fb, bb, cD4, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cA1, ax);
      mzh_mma_store<MT, N2, 4, true, 8, 2>(fa, ba, cD5, sm.x, MZH_LD64, true, nullptr, nullptr, lane, &cA2, ax);
    }
  }
  __syncthreads();
  // ---- E: pol2 / val2 (waves with a head tile), bin 32 of the 33-bin heads (the others)
  if (ht) {
    float* hin = wave == 0 ? sm.hidP : sm.hidV;
    mzh_mma_store<MT, 1, 8, true, 8, 2, true, MzhNoMid, 0, false, false>(fb, bb, cE1, hin, MZH_LD256, false, nullptr,
                                                                       nullptr, lane, &cA1, nullptr, MzhNoMid{}, acc);
    mzh_mma_store<MT, 1, 8, true, 8, 2, true, MzhNoMid, 8, true, true>(fa, ba, cE2, hin, MZH_LD256, false, nullptr,
                                                                     nullptr, lane, &cA2, nullptr, MzhNoMid{}, acc);
  } else if (N2 == 2) {
    mzh_bin32_wave<R>(sm, net, lane);
  }
  __syncthreads();
}

template <int R>
__device__ void mzh_mlp_recurrent(MlpSmem<R>& sm, const MzhNet& net, int wave, int lane) {
  floatx4 fa[16], fb[16];
  float ba[4], bb[4];
  mzh_mlp_fetch12<R>(sm, net, wave, lane, fa, ba, fb, bb);
  if (net.support == 33) {
    mzh_w32_fill<R>(sm, net, threadIdx.x);
    __syncthreads();
  }
  if (net.support == 33)
    mzh_mlp_recurrent_body<R, false, 2, true>(sm, net, wave, lane, fa, ba, fb, bb, net.dyn0_onehot);
  else
    mzh_mlp_recurrent_body<R, false, 1, true>(sm, net, wave, lane, fa, ba, fb, bb, net.dyn0_onehot);
}
