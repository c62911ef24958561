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
#define MZH_THREADS 256

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// fp32 math (networks.py:152-196)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float mzh_expf(float x) {
  if (x < -87.0f) return 0.0f;
  if (x > 88.0f) return __builtin_inff();
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
  return p * __int_as_float((ni + 127) << 23);
}

// _signed_parabolic (networks.py:186-189)
__device__ __forceinline__ float mzh_signed_parabolic(float x) {
  float a = __builtin_fabsf(x);
  float t = 1.00100004673004150390625f + a;
  t = 0.0040000001899898052215576171875f * t;
  t = 1.0f + t;
  t = __builtin_sqrtf(t);
  t = t / 2.0f;
  t = t / 0.001000000047497451305389404296875f;
  float z = t - 500.0f;
  float sg = x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f);
  return sg * (z * z - 1.0f);
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
};

struct MzhNet {
  MzhLayer rep0, rep2, dyn0, dyn2, rwd0, rwd2, pol0, pol2, val0, val2;
  const float* dyn0_onehot;  // [6][256]: dynamic_net.0.weight[:, 64 + a]
  int support;               // 33 or 1
  int in_dim;                // 3N
};

// ------------------------------------------------------------------------------------------
// LDS layout of the MLP block for R roots (R = 16 * MT).  Row strides are 2 (mod 32) dwords so
// the A-fragment ds_read_b32 pattern (row = lane&15, k = 4t + (lane>>4)) is conflict-free.
// ------------------------------------------------------------------------------------------
#define MZH_LD64 66
#define MZH_LD256 258
#define MZH_LDPOL 16
#define MZH_LDSUP 48

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
      const int k = kb * 16 + j * 4 + g;
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          float a = jobs[q].A[(m * 16 + r) * jobs[q].lda + k];
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
        jobs[q].out[row * jobs[q].ldo + col] = v;
      }
    }
  }
}

// normalize_h_state (networks.py:191-196): rows of `src` (stride 66) -> `dst`; one wave per row.
template <int R>
__device__ __forceinline__ void mzh_normalize_rows(const float* src, float* dst, int wave, int lane) {
  for (int row = wave; row < R; row += MZH_THREADS / MZH_WAVE) {
    float v = src[row * MZH_LD64 + lane];
    float mn = v, mx = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float a = __shfl_xor(mn, o);
      float b = __shfl_xor(mx, o);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    float d = (mx - mn) + 9.999999939225290290778502821922302246094e-09f;
    dst[row * MZH_LD64 + lane] = (v - mn) / d;
  }
}

// Heads epilogue: value (wave 0), reward (wave 1, recurrent only), policy softmax (wave 2).
template <int R>
__device__ __forceinline__ void mzh_heads(MlpSmem<R>& sm, int support, bool recurrent, int wave, int lane) {
  if (lane < R) {
    const int row = lane;
    if (wave == 0) {
      sm.value[row] = mzh_logits_to_value(&sm.lval[row * MZH_LDSUP], support);
    } else if (wave == 1) {
      sm.reward[row] = recurrent ? mzh_logits_to_value(&sm.lrwd[row * MZH_LDSUP], support) : 0.0f;
    } else if (wave == 2) {
      float p[MZH_A];
      mzh_softmax6(&sm.lpol[row * MZH_LDPOL], p);
#pragma unroll
      for (int a = 0; a < MZH_A; ++a) sm.pi[row * 8 + a] = p[a];
    }
  }
}

// prediction (networks.py:140-150) on sm.x (normalised latent): policy/value hidden + heads.
template <int R>
__device__ __forceinline__ void mzh_prediction_gemms(MlpSmem<R>& sm, const MzhNet& net, int wave, int lane) {
  constexpr int MT = R / 16;
  // pol0 + val0: 32 tiles, 8 per wave, two chunks of 4
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int id0 = wave * 8 + c * 4;
    const bool val = id0 >= 16;
    const MzhLayer& L = val ? net.val0 : net.pol0;
    MzhJob jobs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      jobs[q] = mzh_job(sm.x, MZH_LD64, L, (id0 + q) & 15, val ? sm.hidV : sm.hidP, MZH_LD256, 1);
    mzh_run_jobs<MT, 4>(jobs, L.kb, nullptr, nullptr, lane);
  }
  __syncthreads();
  // pol2 (1 tile) + val2 (support 33: 3 tiles, support 1: 1 tile)
  {
    int id = wave;
    bool run = id < 1 + net.val2.nt;
    if (run) {
      MzhJob job = id == 0 ? mzh_job(sm.hidP, MZH_LD256, net.pol2, 0, sm.lpol, MZH_LDPOL, 0)
                           : mzh_job(sm.hidV, MZH_LD256, net.val2, id - 1, sm.lval, MZH_LDSUP, 0);
      mzh_run_jobs<MT, 1>(&job, net.pol2.kb, nullptr, nullptr, lane);
    }
  }
  __syncthreads();
}

// initial_inference (networks.py:71-94): sm.x holds obs rows zero-padded to 16*rep0.kb.
template <int R>
__device__ void mzh_mlp_initial(MlpSmem<R>& sm, const MzhNet& net, int wave, int lane) {
  constexpr int MT = R / 16;
  {  // rep0: 16 tiles, 4 per wave
    MzhJob jobs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) jobs[q] = mzh_job(sm.x, MZH_LD64, net.rep0, wave * 4 + q, sm.hidP, MZH_LD256, 1);
    mzh_run_jobs<MT, 4>(jobs, net.rep0.kb, nullptr, nullptr, lane);
  }
  __syncthreads();
  {  // rep2: 4 tiles, 1 per wave
    MzhJob job = mzh_job(sm.hidP, MZH_LD256, net.rep2, wave, sm.hraw, MZH_LD64, 0);
    mzh_run_jobs<MT, 1>(&job, net.rep2.kb, nullptr, nullptr, lane);
  }
  __syncthreads();
  mzh_normalize_rows<R>(sm.hraw, sm.x, wave, lane);
  __syncthreads();
  mzh_prediction_gemms<R>(sm, net, wave, lane);
  mzh_heads<R>(sm, net.support, false, wave, lane);
  __syncthreads();
}

// recurrent_inference (networks.py:96-138): sm.x holds parent latents, sm.act the actions.
// Output: sm.x = normalised new latent, sm.pi / sm.value / sm.reward.
template <int R>
__device__ void mzh_mlp_recurrent(MlpSmem<R>& sm, const MzhNet& net, int wave, int lane) {
  constexpr int MT = R / 16;
  {  // dyn0 (h part, K=64) + one-hot column + bias, relu: 16 tiles, 4 per wave
    MzhJob jobs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) jobs[q] = mzh_job(sm.x, MZH_LD64, net.dyn0, wave * 4 + q, sm.hidP, MZH_LD256, 1);
    mzh_run_jobs<MT, 4>(jobs, net.dyn0.kb, net.dyn0_onehot, sm.act, lane);
  }
  __syncthreads();
  {  // dyn2: 4 tiles, 1 per wave -> un-normalised latent
    MzhJob job = mzh_job(sm.hidP, MZH_LD256, net.dyn2, wave, sm.hraw, MZH_LD64, 0);
    mzh_run_jobs<MT, 1>(&job, net.dyn2.kb, nullptr, nullptr, lane);
  }
  __syncthreads();
  mzh_normalize_rows<R>(sm.hraw, sm.x, wave, lane);
  {  // rwd0 on the UN-normalised latent (networks.py:132): 16 tiles, 4 per wave
    MzhJob jobs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) jobs[q] = mzh_job(sm.hraw, MZH_LD64, net.rwd0, wave * 4 + q, sm.hidR, MZH_LD256, 1);
    mzh_run_jobs<MT, 4>(jobs, net.rwd0.kb, nullptr, nullptr, lane);
  }
  __syncthreads();
  {  // rwd2 (support 33: 3 tiles / 1): waves 0..nt-1
    if (wave < net.rwd2.nt) {
      MzhJob job = mzh_job(sm.hidR, MZH_LD256, net.rwd2, wave, sm.lrwd, MZH_LDSUP, 0);
      mzh_run_jobs<MT, 1>(&job, net.rwd2.kb, nullptr, nullptr, lane);
    }
  }
  mzh_prediction_gemms<R>(sm, net, wave, lane);
  mzh_heads<R>(sm, net.support, true, wave, lane);
  __syncthreads();
}
