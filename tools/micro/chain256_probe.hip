// K = 256 output-layer chain of the latency kernel (csrc/mzh_one.hip one_chain256) in isolation: cycles per
// chain of (a) the DPP form (x in the row layout, v_fmac_f32_dpp row_newbcast, weights from LDS 8 float4 ahead)
// and (b) the broadcast form (x by a uniform-address ds_read_b128 per 4 steps, plain v_fmac_f32), one wave
// alone, three waves on three SIMDs at once (the output-layer phase) and five (waves 0 and 4 share a SIMD).  Weights [64 k4][64 lanes] float4 in LDS.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/chain256_probe.hip -o tools/micro/chain256_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const floatx4 LdsF4;

#define FMAC(j, wi) "v_fmac_f32_dpp %0, %1, %" #wi " row_newbcast:" #j " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void fma16(float& acc, float xv, const float* w) {
  asm("s_nop 1\n\t" FMAC(0, 2) FMAC(1, 3) FMAC(2, 4) FMAC(3, 5) FMAC(4, 6) FMAC(5, 7) FMAC(6, 8) FMAC(7, 9) FMAC(8, 10)
          FMAC(9, 11) FMAC(10, 12) FMAC(11, 13) FMAC(12, 14) FMAC(13, 15) FMAC(14, 16) FMAC(15, 17)
      : "+v"(acc)
      : "v"(xv), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]),
        "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15]));
}

template <int D>
__device__ float chain_dpp(const float* wl, const float* xT, int lane) {
  float xr[16];
  const floatx4* r = reinterpret_cast<const floatx4*>(xT + (lane & 15) * 20);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const floatx4 q = r[m];
    xr[4 * m] = q[0], xr[4 * m + 1] = q[1], xr[4 * m + 2] = q[2], xr[4 * m + 3] = q[3];
  }
  LdsF4* wp = (LdsF4*)(wl + 4 * lane);
  asm volatile("" : "+v"(wp));
  floatx4 wb[D];
#pragma unroll
  for (int i = 0; i < D; ++i) wb[i] = wp[i * 64];
  __builtin_amdgcn_sched_barrier(0);
  float acc = 0.0f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    float ww[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const floatx4 q = wb[(4 * v + i) % D];
      ww[4 * i] = q[0], ww[4 * i + 1] = q[1], ww[4 * i + 2] = q[2], ww[4 * i + 3] = q[3];
    }
    fma16(acc, xr[v], ww);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k4 = 4 * v + i;
      if (k4 + D < 64) wb[k4 % D] = wp[(k4 + D) * 64];
    }
  }
  return acc;
}

template <int D>
__device__ float chain_bcast(const float* wl, const float* x, int lane) {
  LdsF4* wp = (LdsF4*)(wl + 4 * lane);
  LdsF4* xp = (LdsF4*)x;
  asm volatile("" : "+v"(wp), "+v"(xp));
  floatx4 wb[D], xb[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    xb[i] = xp[i];
    wb[i] = wp[i * 64];
  }
  __builtin_amdgcn_sched_barrier(0);
  float acc = 0.0f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const floatx4 q = wb[(4 * v + i) % D], xq = xb[(4 * v + i) % D];
      acc = __builtin_fmaf(xq[0], q[0], acc);
      acc = __builtin_fmaf(xq[1], q[1], acc);
      acc = __builtin_fmaf(xq[2], q[2], acc);
      acc = __builtin_fmaf(xq[3], q[3], acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k4 = 4 * v + i;
      if (k4 + D < 64) {
        wb[k4 % D] = wp[(k4 + D) * 64];
        xb[k4 % D] = xp[k4 + D];
      }
    }
  }
  return acc;
}

// MODE 0: DPP, 1: broadcast; NW waves run the chain (waves 0 .. NW-1), the rest wait at the barrier
template <int MODE, int NW>
__global__ __launch_bounds__(512) void probe(const float* w, float* out, long long* cyc) {
  __shared__ float W[64 * 64 * 4];
  __shared__ float X[320];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int i = t; i < 64 * 64 * 4; i += 512) W[i] = w[i];
  for (int i = t; i < 320; i += 512) X[i] = 1.0f + 1e-3f * i;
  __syncthreads();
  float s = 0.0f;
  long long tot = 0;
  for (int rep = 0; rep < 64; ++rep) {
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (wave < NW) {
      const float y = MODE == 0 ? chain_dpp<8>(W, X, lane) : chain_bcast<8>(W, X, lane);
      X[lane + 64 * (rep & 3)] = y * 1e-9f + 1.0f;  // the next chain's x depends on this one (as in the kernel)
      s += y;
    }
    __syncthreads();
    tot += __builtin_amdgcn_s_memtime() - t0;
  }
  out[t] = s;
  if (t == 0) cyc[MODE * 8 + NW] = tot / 64;
}

int main() {
  float *w, *out;
  long long* cyc;
  hipMalloc(&w, 64 * 64 * 16);
  hipMalloc(&out, 512 * 4);
  hipMalloc(&cyc, 16 * 8);
  hipMemset(w, 0, 64 * 64 * 16);
  long long h[16] = {};
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((probe<0, 0>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipLaunchKernelGGL((probe<0, 1>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipLaunchKernelGGL((probe<0, 3>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipLaunchKernelGGL((probe<1, 1>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipLaunchKernelGGL((probe<1, 3>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipLaunchKernelGGL((probe<0, 5>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipLaunchKernelGGL((probe<1, 5>), dim3(1), dim3(512), 0, 0, w, out, cyc);
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  }
  printf("{\"empty\": %lld, \"dpp_1wave\": %lld, \"dpp_3waves\": %lld, \"bcast_1wave\": %lld, \"bcast_3waves\": %lld, "
         "\"dpp_5waves\": %lld, \"bcast_5waves\": %lld, "
         "\"unit\": \"s_memtime ticks per 256-step chain incl. two barriers\"}\n",
         h[0], h[1], h[3], h[9], h[11], h[5], h[13]);
  return 0;
}
