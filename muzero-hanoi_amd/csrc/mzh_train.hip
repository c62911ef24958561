// mzh_train.hip -- fused MuZero training update on gfx950: Muzero._update (Muzero.py:209-274)
// followed by MuZeroNet.update / torch.optim.Adam (networks.py:69,118-122) in two launches.
//
//   mzt_rows_kernel<R, SUP>   one 256-thread workgroup per R transitions.  The 5-step unrolled
//       forward (represent; per step prediction, dynamics, reward; networks.py:124-196) and its
//       whole backward pass (MSE value / reward terms through the softmax-expectation and signed
//       parabolic transforms, soft-target cross-entropy for the policy, the 0.5 latent-gradient
//       hook, the min/max normalisation, importance weights and the 1/U loss hook) run in
//       registers and LDS; every Linear layer's input X and output-gradient GY is written to a
//       scratch area in HBM.  Each GEMV reads whichever of torch's [out][in] weight or its
//       transposed copy [in][out] is contiguous along the threads: thread-per-output for the
//       256-wide hidden layers, split-K (thread = output x input chunk, partials summed through
//       LDS) for the narrow 64 / 33 / 6-wide layers.
//   mzt_grad_adam_kernel      one workgroup per 16x16 weight tile of the 10 Linear layers:
//       dW = GY^T X over all B*U (or B) rows as a v_mfma_f32_16x16x4_f32 chain (4 waves split the
//       rows, reduced in LDS), bias sums, then Adam (torch's update order: lerp of the first
//       moment, second moment, sqrt / bias-correction / eps, addcdiv) in place on the torch
//       parameter and state tensors, and the transposed weight copy refreshed.
//
// The arithmetic is fp32 like torch's; sums run in other orders than hipBLASLt / torch-CPU, so
// results agree with the reference to fp32 rounding (tests/test_training.py), not bit for bit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mzh_train.h"

namespace {

constexpr int H = 64, F = 256, A = 6;

// all-lane wave reductions without LDS: DPP within rows of 16 (xor 1, xor 2, half-mirror, mirror),
// then v_permlane16_swap / v_permlane32_swap across rows
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float swap16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float swap32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
template <class Op>
__device__ __forceinline__ float wave_reduce(float v, Op op) {
  v = op(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp<0x141>(v));  // row_half_mirror
  v = op(v, dpp<0x140>(v));  // row_mirror
  v = op(v, swap16(v));
  v = op(v, swap32(v));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float a, float b) { return a + b; });
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float a, float b) { return fmaxf(a, b); });
}
__device__ __forceinline__ float wave_min(float v) {
  return wave_reduce(v, [](float a, float b) { return fminf(a, b); });
}

// first lane index holding `v` among lanes where `hit` (ties -> lowest index, torch-CPU's choice)
__device__ __forceinline__ int wave_first(bool hit) {
  const unsigned long long m = __ballot(hit);
  return m ? __ffsll((long long)m) - 1 : 0;
}
__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// signed parabolic transform of networks.py:185-189, op by op in fp32
struct Parab {
  float x, e, z, s;
};
__device__ __forceinline__ Parab parab_fwd(float x) {
  Parab p;
  p.x = x;
  p.s = sgnf(x);
  const float a = fabsf(x);
  const float b = 1.001f + a;     // eps + 1 + |x|  (eps + 1 folded as in Python)
  const float c = 0.004f * b;     // 4 * eps * (...)
  const float d = 1.0f + c;
  p.e = sqrtf(d);
  const float f = p.e / 2.0f;
  const float g = f / 0.001f;
  p.z = g - 500.0f;               // - 1 / 2 / eps
  return p;
}
__device__ __forceinline__ float parab_out(const Parab& p) { return p.s * (p.z * p.z - 1.0f); }
// d out / d x times gout, through torch's autograd chain (sign' = 0, |x|' = sign(x))
__device__ __forceinline__ float parab_bwd(const Parab& p, float gout) {
  const float gr = gout * p.s;
  const float gz = 2.0f * p.z * gr;
  const float gf = gz / 0.001f;
  const float ge = gf / 2.0f;
  const float gd = ge / (2.0f * p.e);
  const float gb = 0.004f * gd;
  return gb * p.s;
}

// ------------------------------------------------------------------------------------------
// k-major GEMV pieces.  Every Linear layer, in both directions, is read from whichever of torch's
// [out][in] weight or its transposed copy [in][out_pad] has the OUTPUT index contiguous ("k-major":
// element (k, c) at W[k * ldw + c], rows 16-byte aligned).  Thread t -> (column group cg = t % C4
// of 4 outputs, input chunk q = t / C4 of Q chunks): one float4 weight load feeds 4 R FMAs, and
// the Q partial sums of each output are added through LDS by kcomb after a barrier.
template <int R, int C4, int Q>
__device__ __forceinline__ void kpart(const float* __restrict__ W, int ldw, int K, const float* X, int ldx,
                                      float* P) {
  const int t = threadIdx.x;
  if (t >= C4 * Q) return;
  const int cg = t % C4, q = t / C4;
  const int cs = (K + Q - 1) / Q;
  const int k0 = q * cs, k1 = min(K, k0 + cs);
  float4 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
  for (int k = k0; k < k1; ++k) {
    const float4 w = *(const float4*)(W + (size_t)k * ldw + 4 * cg);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float x = X[r * ldx + k];
      acc[r].x = fmaf(w.x, x, acc[r].x);
      acc[r].y = fmaf(w.y, x, acc[r].y);
      acc[r].z = fmaf(w.z, x, acc[r].z);
      acc[r].w = fmaf(w.w, x, acc[r].w);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) *(float4*)(P + (q * R + r) * (4 * C4) + 4 * cg) = acc[r];
}
// the same with float2 loads for a weight whose rows are only 8-byte aligned (dynamics layer 1,
// [256][70]); C2 column pairs
template <int R, int C2, int Q>
__device__ __forceinline__ void kpart2(const float* __restrict__ W, int ldw, int K, const float* X, int ldx,
                                       float* P) {
  const int t = threadIdx.x;
  if (t >= C2 * Q) return;
  const int cg = t % C2, q = t / C2;
  const int cs = (K + Q - 1) / Q;
  const int k0 = q * cs, k1 = min(K, k0 + cs);
  float2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = make_float2(0.f, 0.f);
#pragma unroll 4
  for (int k = k0; k < k1; ++k) {
    const float2 w = *(const float2*)(W + (size_t)k * ldw + 2 * cg);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float x = X[r * ldx + k];
      acc[r].x = fmaf(w.x, x, acc[r].x);
      acc[r].y = fmaf(w.y, x, acc[r].y);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) *(float2*)(P + (q * R + r) * (2 * C2) + 2 * cg) = acc[r];
}
// sum of the Q partials of output c of row r (fixed order q = 0..Q-1)
template <int R, int Q>
__device__ __forceinline__ float kcomb(const float* P, int ldp, int r, int c) {
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < Q; ++q) v += P[(q * R + r) * ldp + c];
  return v;
}

// threads of a row-kernel workgroup: 512, two waves per SIMD (measured against 256, one per SIMD)
constexpr int RNT = 512;

// LDS plan of the rows kernel (floats), U steps, R rows
constexpr int RED_PER_ROW = 12 * RNT;  // split-K partials: 3 areas x (RNT / 64 chunks x 256 outputs)
template <int R>
struct RowLds {
  // multiple of 4 floats: the per-step activation rows are read as float4
  __device__ __host__ static int per_step() { return (R * (4 * F + H + 8 + 48 + 48) + 2 * R + 3) & ~3; }
  __device__ __host__ static int fixed() {
    return R * (32 + F + H + H + H + H + 8 + 48 + 48 + 4 * F + RED_PER_ROW) + 8 * R + 64;
  }
  __device__ __host__ static size_t bytes(int U) { return sizeof(float) * (size_t)(fixed() + U * per_step()); }
};

template <int R, int SUP>
__global__ __launch_bounds__(RNT, 1) void mzt_rows_kernel(MztRowParams p) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int U = p.U, B = p.B;
  const int b0 = blockIdx.x * R;
  constexpr int LDS_SUP = 48;
  constexpr int LD_GS = SUP > 1 ? 48 : 16;  // padded widths of the GY logit arrays (kernel 2 reads 16-col tiles)
  constexpr int LDV = (SUP + 3) & ~3;       // row stride of the value / reward layer-2 transposed copies
  constexpr int CV = LDV / 4;

  // ---- LDS carve-up
  float* x0 = lds;                    // [R][32]
  float* repa = x0 + R * 32;          // [R][F]
  float* h = repa + R * F;            // [R][H] current normalised latent h_t
  float* gh = h + R * H;              // [R][H] gradient of h_{t+1} from later steps
  float* ghp = gh + R * H;            // [R][H] gradient of h'_{t+1}
  float* hp0 = ghp + R * H;           // [R][H] representation output before normalisation
  float* glp = hp0 + R * H;           // [R][8]
  float* glv = glp + R * 8;           // [R][48]
  float* glr = glv + R * 48;          // [R][48]
  float* gph = glr + R * 48;          // [R][F] policy hidden pre-activation gradient
  float* gvh = gph + R * F;
  float* grh = gvh + R * F;
  float* gdh = grh + R * F;
  float* red = gdh + R * F;           // split-K partials, RED_PER_ROW * R floats
  float* red1 = red + R * 4 * RNT;    // second and third partial areas (4 RNT R floats each)
  float* red2 = red + R * 8 * RNT;
  float* rowf = red + R * RED_PER_ROW;  // [8][R] per-row scalars: 0 v_loss, 1 r_loss, 2 p_loss, 3 g_b
  int* acts = (int*)(rowf + 8 * R);   // [64] actions (R*U <= 64)
  float* st = (float*)(acts + 64);    // per-step block
  const int PS = RowLds<R>::per_step();
  auto s_ap = [&](int t) { return st + t * PS; };                 // [R][F]
  auto s_av = [&](int t) { return st + t * PS + R * F; };
  auto s_ad = [&](int t) { return st + t * PS + 2 * R * F; };
  auto s_ar = [&](int t) { return st + t * PS + 3 * R * F; };
  auto s_hp = [&](int t) { return st + t * PS + 4 * R * F; };     // [R][H]  h'_{t+1}
  auto s_lp = [&](int t) { return st + t * PS + 4 * R * F + R * H; };              // [R][8]
  auto s_lv = [&](int t) { return st + t * PS + 4 * R * F + R * H + R * 8; };      // [R][48]
  auto s_lr = [&](int t) { return st + t * PS + 4 * R * F + R * H + R * 56; };     // [R][48]
  auto s_vr = [&](int t) { return st + t * PS + 4 * R * F + R * H + R * 104; };    // [2][R] v_t, r_t

  const MztNet& n = p.n;
  const MztScratch& s = p.s;
  auto rowb = [&](int r) { return min(b0 + r, B - 1); };
  auto valid = [&](int r) { return b0 + r < B; };

  // ---- inputs
  for (int i = tid; i < R * 32; i += RNT) {
    const int r = i >> 5, k = i & 31;
    const float v = k < p.in_dim ? p.obs[(size_t)rowb(r) * p.in_dim + k] : 0.f;
    x0[i] = v;
    if (valid(r)) s.x0[(size_t)(b0 + r) * 32 + k] = v;
  }
  for (int i = tid; i < R * U; i += RNT) acts[i] = (int)p.actions[(size_t)rowb(i / U) * U + (i % U)];
  if (tid < R) {
    const int r = tid;
    rowf[0 * R + r] = rowf[1 * R + r] = rowf[2 * R + r] = 0.f;
    const float w = p.w ? p.w[rowb(r)] : 1.0f;
    rowf[3 * R + r] = valid(r) ? ((1.0f / (float)U) / (float)B) * w : 0.f;
  }
  __syncthreads();

  // ---- representation: hidden, output, normalise
  kpart<R, 64, RNT / 64>(n.rep1T, F, p.in_dim, x0, 32, red);
  __syncthreads();
  for (int i = tid; i < R * F; i += RNT) {
    const int r = i / F, c = i - r * F;
    const float a = fmaxf(kcomb<R, RNT / 64>(red, F, r, c) + n.rep1b[c], 0.f);
    repa[i] = a;
    if (valid(r)) s.repa[(size_t)(b0 + r) * F + c] = a;
  }
  __syncthreads();
  kpart<R, 16, RNT / 16>(n.rep2T, H, F, repa, F, red);
  __syncthreads();
  for (int i = tid; i < R * H; i += RNT) {
    const int r = i / H, c = i - r * H;
    hp0[i] = kcomb<R, RNT / 16>(red, H, r, c) + n.rep2b[c];
  }
  __syncthreads();
  for (int r = wave; r < R; r += RNT / 64) {
    const float v = hp0[r * H + lane];
    const float mn = wave_min(v), mx = wave_max(v);
    const float y = (v - mn) / ((mx - mn) + 1e-8f);
    h[r * H + lane] = y;
    if (valid(r)) s.h[((size_t)(b0 + r) * U + 0) * H + lane] = y;
  }
  __syncthreads();

  // ---- unrolled forward
  for (int t = 0; t < U; ++t) {
    float* ap = s_ap(t);
    float* av = s_av(t);
    float* ad = s_ad(t);
    float* ar = s_ar(t);
    float* hp = s_hp(t);
    float* lp = s_lp(t);
    float* lv = s_lv(t);
    float* lr = s_lr(t);
    float* vr = s_vr(t);
    // S1: policy / value / dynamics hidden layers, all on h_t (dynamics' one-hot column added below)
    kpart<R, 64, RNT / 64>(n.pol1T, F, H, h, H, red);
    kpart<R, 64, RNT / 64>(n.val1T, F, H, h, H, red1);
    kpart<R, 64, RNT / 64>(n.dyn1T, F, H, h, H, red2);
    __syncthreads();
    for (int i = tid; i < R * F; i += RNT) {
      const int r = i / F, c = i - r * F;
      const float a1 = fmaxf(kcomb<R, RNT / 64>(red, F, r, c) + n.pol1b[c], 0.f);
      const float a2 = fmaxf(kcomb<R, RNT / 64>(red1, F, r, c) + n.val1b[c], 0.f);
      const float a3 = fmaxf((kcomb<R, RNT / 64>(red2, F, r, c) + n.dyn1T[(H + acts[r * U + t]) * F + c]) + n.dyn1b[c], 0.f);
      ap[i] = a1;
      av[i] = a2;
      ad[i] = a3;
      if (valid(r)) {
        const size_t m = (size_t)(b0 + r) * U + t;
        s.ap[m * F + c] = a1;
        s.av[m * F + c] = a2;
        s.ad[m * F + c] = a3;
      }
    }
    __syncthreads();
    // S2: policy logits, value logits, dynamics output h'_{t+1}: split-K over the transposed copies
    kpart<R, 2, RNT / 8>(n.pol2T, 8, F, ap, F, red);
    kpart<R, CV, RNT / CV < 64 ? RNT / CV : 64>(n.val2T, LDV, F, av, F, red1);
    kpart<R, 16, RNT / 16>(n.dyn2T, H, F, ad, F, red2);
    __syncthreads();
    for (int i = tid; i < R * H; i += RNT) {
      const int r = i / H, c = i - r * H;
      hp[i] = kcomb<R, RNT / 16>(red2, H, r, c) + n.dyn2b[c];
    }
    for (int i = tid; i < R * SUP; i += RNT) {
      const int r = i / SUP, c = i - r * SUP;
      lv[r * LDS_SUP + c] = kcomb<R, (RNT / CV < 64 ? RNT / CV : 64)>(red1, LDV, r, c) + n.val2b[c];
    }
    for (int i = tid; i < R * A; i += RNT) {
      const int r = i / A, c = i - r * A;
      lp[r * 8 + c] = kcomb<R, RNT / 8>(red, 8, r, c) + n.pol2b[c];
    }
    __syncthreads();
    // S3: normalise h'_{t+1} -> h_{t+1} (one wave per row), reward hidden layer on h'_{t+1}
    for (int r = wave; r < R; r += RNT / 64) {
      const float v = hp[r * H + lane];
      const float mn = wave_min(v), mx = wave_max(v);
      const float y = (v - mn) / ((mx - mn) + 1e-8f);
      h[r * H + lane] = y;
      if (valid(r)) {
        const size_t m = (size_t)(b0 + r) * U + t;
        s.hp[m * H + lane] = v;
        if (t + 1 < U) s.h[(m + 1) * H + lane] = y;
      }
    }
    kpart<R, 64, RNT / 64>(n.rwd1T, F, H, hp, H, red);
    __syncthreads();
    for (int i = tid; i < R * F; i += RNT) {
      const int r = i / F, c = i - r * F;
      const float a = fmaxf(kcomb<R, RNT / 64>(red, F, r, c) + n.rwd1b[c], 0.f);
      ar[i] = a;
      if (valid(r)) s.ar[((size_t)(b0 + r) * U + t) * F + c] = a;
    }
    __syncthreads();
    // S4: reward logits
    kpart<R, CV, RNT / CV < 64 ? RNT / CV : 64>(n.rwd2T, LDV, F, ar, F, red);
    __syncthreads();
    for (int i = tid; i < R * SUP; i += RNT) {
      const int r = i / SUP, c = i - r * SUP;
      lr[r * LDS_SUP + c] = kcomb<R, (RNT / CV < 64 ? RNT / CV : 64)>(red, LDV, r, c) + n.rwd2b[c];
    }
    __syncthreads();
    // S5: heads and loss terms; task = (head, row), heads: 0 value, 1 reward, 2 policy
    for (int task = wave; task < 3 * R; task += RNT / 64) {
      const int hd = task / R, r = task - hd * R;
      const int bb = rowb(r);
      if (hd < 2) {
        const float* lg = hd == 0 ? lv + r * LDS_SUP : lr + r * LDS_SUP;
        float val;
        if (SUP > 1) {
          const float l = lane < SUP ? lg[lane] : -INFINITY;
          const float mx = wave_max(l);
          const float e = lane < SUP ? expf(l - mx) : 0.f;
          const float se = wave_sum(e);
          const float pk = e / se;
          const float x = wave_sum(lane < SUP ? pk * (float)(lane - (SUP - 1) / 2) : 0.f);
          val = parab_out(parab_fwd(x));
        } else {
          val = lg[0];
        }
        const float target = hd == 0 ? p.returns[(size_t)bb * U + t] : p.rwds[(size_t)bb * U + t];
        const float d = val - target;
        if (lane == 0) {
          vr[hd * R + r] = val;
          rowf[hd * R + r] += d * d;
          if (hd == 0 && t == 0 && p.new_prio && valid(r)) p.new_prio[b0 + r] = fabsf(d);
        }
      } else {
        const float l = lane < A ? lp[r * 8 + lane] : -INFINITY;
        const float mx = wave_max(l);
        const float se = wave_sum(lane < A ? expf(l - mx) : 0.f);
        const float lse = mx + logf(se);
        const float pi = lane < A ? p.pi[((size_t)bb * U + t) * A + lane] : 0.f;
        const float ce = -wave_sum(lane < A ? pi * (l - lse) : 0.f);
        if (lane == 0) rowf[2 * R + r] += ce;
      }
    }
    __syncthreads();
  }

  // ---- backward through the unroll
  for (int i = tid; i < R * H; i += RNT) gh[i] = 0.f;
  __syncthreads();
  for (int t = U - 1; t >= 0; --t) {
    const float* ap = s_ap(t);
    const float* av = s_av(t);
    const float* ad = s_ad(t);
    const float* ar = s_ar(t);
    const float* hp = s_hp(t);
    const float* lp = s_lp(t);
    const float* lv = s_lv(t);
    const float* lr = s_lr(t);
    const float* vr = s_vr(t);
    // B1: head gradients (tasks 0..3R-1) and the normalisation backward of h_{t+1} with the
    //     0.5 hook (tasks 3R..4R-1)
    for (int task = wave; task < 4 * R; task += RNT / 64) {
      const int hd = task / R, r = task - hd * R;
      const int bb = rowb(r);
      const size_t m = (size_t)(b0 + r) * U + t;
      const float g = rowf[3 * R + r];
      if (hd < 2) {
        const float* lg = hd == 0 ? lv + r * LDS_SUP : lr + r * LDS_SUP;
        const float target = hd == 0 ? p.returns[(size_t)bb * U + t] : p.rwds[(size_t)bb * U + t];
        const float gval = 2.0f * (vr[hd * R + r] - target) * g;  // mse_loss backward
        float gl;
        if (SUP > 1) {
          const float l = lane < SUP ? lg[lane] : -INFINITY;
          const float mx = wave_max(l);
          const float e = lane < SUP ? expf(l - mx) : 0.f;
          const float se = wave_sum(e);
          const float pk = e / se;
          const float sk = (float)(lane - (SUP - 1) / 2);
          const float x = wave_sum(lane < SUP ? pk * sk : 0.f);
          const float gx = parab_bwd(parab_fwd(x), gval);
          const float gp = gx * sk;                       // sum / mul backward
          const float dot = wave_sum(lane < SUP ? gp * pk : 0.f);
          gl = lane < SUP ? pk * (gp - dot) : 0.f;         // softmax backward
        } else {
          gl = lane == 0 ? gval : 0.f;
        }
        float* gdst = hd == 0 ? glv : glr;
        if (lane < 48) gdst[r * 48 + lane] = gl;
        float* gg = hd == 0 ? s.g_lv : s.g_lr;
        if (valid(r) && lane < LD_GS) gg[m * LD_GS + lane] = gl;
      } else if (hd == 2) {
        const float l = lane < A ? lp[r * 8 + lane] : -INFINITY;
        const float mx = wave_max(l);
        const float se = wave_sum(lane < A ? expf(l - mx) : 0.f);
        const float lse = mx + logf(se);
        const float pi = lane < A ? p.pi[((size_t)bb * U + t) * A + lane] : 0.f;
        const float spi = wave_sum(pi);
        const float gl = lane < A ? g * (expf(l - lse) * spi - pi) : 0.f;  // soft-target CE backward
        if (lane < 8) glp[r * 8 + lane] = gl;
        if (valid(r) && lane < 16) s.g_lp[m * 16 + lane] = gl;
      } else {
        // y = (h' - mn) / D, D = (mx - mn) + 1e-8; incoming gradient 0.5 * gh (the register_hook)
        const float v = hp[r * H + lane];
        const float gy = gh[r * H + lane] * 0.5f;
        const float mn = wave_min(v), mxv = wave_max(v);
        const float D = (mxv - mn) + 1e-8f;
        const float sub = v - mn;
        const float gs = gy / D;
        const float gD = -wave_sum(gy * sub / (D * D));
        const float gmn = -wave_sum(gs) - gD;
        const int imn = wave_first(v == mn), imx = wave_first(v == mxv);
        float gv = gs;
        if (lane == imn) gv += gmn;
        if (lane == imx) gv += gD;
        ghp[r * H + lane] = gv;
      }
    }
    __syncthreads();
    // B2: hidden-layer gradients of the reward, value and policy heads through torch's [out][256]
    //     layer-2 weights (k-major over the logits)
    kpart<R, 64, RNT / 64>(n.rwd2, F, SUP, glr, 48, red);
    kpart<R, 64, RNT / 64>(n.val2, F, SUP, glv, 48, red1);
    kpart<R, 64, RNT / 64>(n.pol2, F, A, glp, 8, red2);
    __syncthreads();
    for (int i = tid; i < R * F; i += RNT) {
      const int r = i / F, c = i - r * F;
      const float g1 = ar[i] > 0.f ? kcomb<R, RNT / 64>(red, F, r, c) : 0.f;
      const float g2 = av[i] > 0.f ? kcomb<R, RNT / 64>(red1, F, r, c) : 0.f;
      const float g3 = ap[i] > 0.f ? kcomb<R, RNT / 64>(red2, F, r, c) : 0.f;
      grh[i] = g1;
      gvh[i] = g2;
      gph[i] = g3;
      if (valid(r)) {
        const size_t m = (size_t)(b0 + r) * U + t;
        s.g_r[m * F + c] = g1;
        s.g_v[m * F + c] = g2;
        s.g_p[m * F + c] = g3;
      }
    }
    __syncthreads();
    // B3: h'_{t+1} gradient += reward layer-1 backward (torch's [256][64]: k-major over the hidden units)
    kpart<R, 16, RNT / 16>(n.rwd1, H, F, grh, F, red);
    __syncthreads();
    for (int i = tid; i < R * H; i += RNT) {
      const int r = i / H, c = i - r * H;
      const float v = ghp[i] + kcomb<R, RNT / 16>(red, H, r, c);
      ghp[i] = v;
      if (valid(r)) s.g_hp[((size_t)(b0 + r) * U + t) * H + c] = v;
    }
    __syncthreads();
    // B4: dynamics hidden gradient (torch's [64][256] layer-2 weight)
    kpart<R, 64, RNT / 64>(n.dyn2, F, H, ghp, H, red);
    __syncthreads();
    for (int i = tid; i < R * F; i += RNT) {
      const int r = i / F, c = i - r * F;
      const float g = ad[i] > 0.f ? kcomb<R, RNT / 64>(red, F, r, c) : 0.f;
      gdh[i] = g;
      if (valid(r)) s.g_d[((size_t)(b0 + r) * U + t) * F + c] = g;
    }
    __syncthreads();
    // B5: gradient of h_t = dynamics + value + policy layer-1 backward (latent columns only)
    kpart2<R, 32, RNT / 32>(n.dyn1, H + A, F, gdh, F, red);
    kpart<R, 16, RNT / 16>(n.val1, H, F, gvh, F, red1);
    kpart<R, 16, RNT / 16>(n.pol1, H, F, gph, F, red2);
    __syncthreads();
    for (int i = tid; i < R * H; i += RNT) {
      const int r = i / H, c = i - r * H;
      gh[i] = (kcomb<R, RNT / 32>(red, H, r, c) + kcomb<R, RNT / 16>(red1, H, r, c)) + kcomb<R, RNT / 16>(red2, H, r, c);
    }
    __syncthreads();
  }

  // ---- representation backward: normalisation of h_0 (no hook), then the output layer
  for (int r = wave; r < R; r += RNT / 64) {
    const float v = hp0[r * H + lane];
    const float gy = gh[r * H + lane];
    const float mn = wave_min(v), mxv = wave_max(v);
    const float D = (mxv - mn) + 1e-8f;
    const float sub = v - mn;
    const float gs = gy / D;
    const float gD = -wave_sum(gy * sub / (D * D));
    const float gmn = -wave_sum(gs) - gD;
    const int imn = wave_first(v == mn), imx = wave_first(v == mxv);
    float gv = gs;
    if (lane == imn) gv += gmn;
    if (lane == imx) gv += gD;
    ghp[r * H + lane] = gv;
    if (valid(r)) s.g_h0p[(size_t)(b0 + r) * H + lane] = gv;
  }
  __syncthreads();
  kpart<R, 64, RNT / 64>(n.rep2, F, H, ghp, H, red);
  __syncthreads();
  for (int i = tid; i < R * F; i += RNT) {
    const int r = i / F, c = i - r * F;
    const float g = repa[i] > 0.f ? kcomb<R, RNT / 64>(red, F, r, c) : 0.f;
    if (valid(r)) s.g_rep[(size_t)(b0 + r) * F + c] = g;
  }
  if (tid < R && valid(tid)) {
    const int r = tid;
    p.row_loss[(size_t)(b0 + r) * 3 + 0] = rowf[0 * R + r];
    p.row_loss[(size_t)(b0 + r) * 3 + 1] = rowf[1 * R + r];
    p.row_loss[(size_t)(b0 + r) * 3 + 2] = rowf[2 * R + r];
  }
}

// ------------------------------------------------------------------------------------------
// weight gradients + Adam: one workgroup per 16x16 tile of one Linear layer
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void adam(float* pp, float* mm, float* vv, size_t i, float g, const MztGradParams& P) {
  float m = mm[i], v = vv[i];
  m = m + (1.0f - P.beta1) * (g - m);           // exp_avg.lerp_(grad, 1 - beta1)
  v = v * P.beta2 + (1.0f - P.beta2) * (g * g);  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / P.bc2_sqrt + P.eps;
  pp[i] = pp[i] + (-P.step_size) * (m / denom);
  mm[i] = m;
  vv[i] = v;
}

constexpr int NW2 = 16;  // waves per weight tile: they split the B*U rows
__global__ __launch_bounds__(64 * NW2) void mzt_grad_adam_kernel(MztGradParams P) {
  constexpr int NP = 4 * NW2;  // bias row classes (16 columns x NP)
  __shared__ float red[NW2][16][17];
  __shared__ float bred[NP][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int li = 0;
  while (li < 9 && (int)blockIdx.x >= P.L[li + 1].tile0) ++li;
  const MztGradLayer& L = P.L[li];
  const int tile = blockIdx.x - L.tile0;
  const int ob = tile / L.nkb, kb = tile - ob * L.nkb;
  const int o0 = ob * 16, k0 = kb * 16;
  const int col = lane & 15, sub = lane >> 4;

  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const int oc = o0 + col, kc = k0 + col;
  // one-hot action columns (dynamics layer 1, k >= 64) are generated, not loaded; 64 is a multiple
  // of 16 so a tile is either all one-hot or all X
  const bool onehot = L.onehot_from >= 0 && k0 >= L.onehot_from;
  const int act_col = kc - L.onehot_from;
  const bool kin = kc < L.in;
  // rows m = 4 (wave + NW2 i) + sub; loads batched ahead of the MFMA chain
  constexpr int UNR = 8, STEP = 4 * NW2;
  for (int base = 4 * wave; base < L.M; base += STEP * UNR) {
    float a[UNR], b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int m = base + STEP * u + sub;
      const bool ok = m < L.M;
      a[u] = ok ? L.GY[(size_t)m * L.ldg + oc] : 0.f;
      if (onehot)
        b[u] = (ok && (int)P.actions[m] == act_col) ? 1.f : 0.f;
      else
        b[u] = (ok && kin) ? L.X[(size_t)m * L.ldx + kc] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][4 * sub + r][col] = acc[r];
  if (kb == 0) {
    // bias: sum of GY column o0 + (tid & 15) over rows m = tid >> 4 (mod NP), UNR independent sums
    const int i = tid & 15, part = tid >> 4;
    float sb[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) sb[u] = 0.f;
    for (int m = part; m < L.M; m += NP * UNR) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int mm = m + NP * u;
        sb[u] += mm < L.M ? L.GY[(size_t)mm * L.ldg + o0 + i] : 0.f;
      }
    }
    float t = 0.f;
#pragma unroll
    for (int u = 0; u < UNR; ++u) t += sb[u];
    bred[part][i] = t;
  }
  __syncthreads();
  if (tid < 256) {
    const int i = tid >> 4, j = tid & 15;
    const int o = o0 + i, k = k0 + j;
    if (o < L.out && k < L.in) {
      float g = 0.f;
#pragma unroll
      for (int w = 0; w < NW2; ++w) g += red[w][i][j];
      const size_t idx = (size_t)o * L.in + k;
      adam(L.W, L.mW, L.vW, idx, g, P);
      L.WT[(size_t)k * L.ldwt + o] = L.W[idx];
    }
  }
  if (kb == 0 && tid < 16 && o0 + tid < L.out) {
    float g = 0.f;
    for (int part = 0; part < NP; ++part) g += bred[part][tid];
    adam(L.b, L.mb, L.vb, o0 + tid, g, P);
  }
}

__global__ void mzt_transpose_kernel(const float* W, float* WT, int out, int in, int ldwt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ldwt * in) {
    const int k = i / ldwt, o = i - k * ldwt;
    WT[i] = o < out ? W[(size_t)o * in + k] : 0.f;  // pad columns stay zero
  }
}

template <int R, int SUP>
hipError_t launch_rows(const MztRowParams& p, hipStream_t stream) {
  const size_t smem = RowLds<R>::bytes(p.U);
  auto kern = mzt_rows_kernel<R, SUP>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((p.B + R - 1) / R), dim3(RNT), smem, stream, p);
  return hipGetLastError();
}

}  // namespace

size_t mzt_rows_smem_bytes(int rows, int U) { return rows == 1 ? RowLds<1>::bytes(U) : RowLds<2>::bytes(U); }

hipError_t mzt_launch_rows(int rows, int support, const MztRowParams& p, hipStream_t stream) {
  if (support == 33) return rows == 1 ? launch_rows<1, 33>(p, stream) : launch_rows<2, 33>(p, stream);
  return rows == 1 ? launch_rows<1, 1>(p, stream) : launch_rows<2, 1>(p, stream);
}

hipError_t mzt_launch_grad_adam(const MztGradParams& P, int n_tiles, hipStream_t stream) {
  hipLaunchKernelGGL(mzt_grad_adam_kernel, dim3(n_tiles), dim3(64 * NW2), 0, stream, P);
  return hipGetLastError();
}

hipError_t mzt_launch_transpose(const float* W, float* WT, int out, int in, int ldwt, hipStream_t stream) {
  const int n = ldwt * in;
  hipLaunchKernelGGL(mzt_transpose_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, W, WT, out, in, ldwt);
  return hipGetLastError();
}
