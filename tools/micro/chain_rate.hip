// Microbenchmark: the search MLP's NJ=4 x MT=2 x KB=4 MFMA chunk (128 v_mfma_f32_16x16x4_f32 per
// wave) with its operand traffic switched on piece by piece: A from LDS (ds_read_b128, one k-block
// ahead), B from a 16-fragment register buffer refilled from L2 (ring), the epilogue's LDS stores.
// One wave per SIMD, 256 workgroups.  Diagnostic only, not shipped.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <bool LDSA, bool RING, bool EPI, int NJ, int KB>
__global__ __launch_bounds__(256, 1) void k_chain(const float4* w, float* out, unsigned long long* ticks, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[32 * 260];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < 32 * 260; i += 256) lds[i] = 1e-3f * (i & 15);
  __syncthreads();
  floatx4 f[16];
  for (int s = 0; s < 16; ++s) {
    float4 t = w[(wave * 16 + s) * 64 + lane];
    f[s] = floatx4{t.x, t.y, t.z, t.w};
  }
  float* outp = lds + wave * 64;
  const float* arow = lds + r * 68 + 4 * g;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  floatx4 keep = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    floatx4 acc[NJ][2];
#pragma unroll
    for (int q = 0; q < NJ; ++q) acc[q][0] = acc[q][1] = floatx4{0, 0, 0, 0};
    floatx4 a[2][2];
    if (LDSA) {
#pragma unroll
      for (int m = 0; m < 2; ++m) a[0][m] = *reinterpret_cast<const floatx4*>(arow + m * 16 * 68);
    } else {
      a[0][0] = a[0][1] = a[1][0] = a[1][1] = floatx4{1e-3f * lane, 2e-3f, 3e-3f, 4e-3f};
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if (LDSA && kb + 1 < KB) {
#pragma unroll
        for (int m = 0; m < 2; ++m) a[(kb + 1) & 1][m] = *reinterpret_cast<const floatx4*>(arow + m * 16 * 68 + (kb + 1) * 16);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < NJ; ++q)
#pragma unroll
          for (int m = 0; m < 2; ++m)
            acc[q][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kb & 1][m][j], f[q * KB + kb][j], acc[q][m], 0, 0, 0);
      if (RING) {
#pragma unroll
        for (int q = 0; q < NJ; ++q) {
          float4 t = w[((it & 7) * 64 + wave * 16 + q * KB + kb) * 64 + lane];
          f[q * KB + kb] = floatx4{t.x, t.y, t.z, t.w};
        }
      }
    }
    if (EPI) {
#pragma unroll
      for (int q = 0; q < NJ; ++q)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = acc[q][m][i] + 0.5f;
            outp[(m * 16 + g * 4 + i) * 260 + q * 16 + 4 * (r & 3) + (r >> 2)] = v > 0.f ? v : 0.f;
          }
    } else {
#pragma unroll
      for (int q = 0; q < NJ; ++q) keep += acc[q][0] + acc[q][1];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = keep[0] + keep[1] + keep[2] + keep[3];
  if (lane == 0) ticks[blockIdx.x * 4 + wave] = t1 - t0;
}

template <bool LDSA, bool RING, bool EPI, int NJ, int KB>
void run(const char* name, const float4* w, float* out, unsigned long long* ticks) {
  const int iters = 2000;
  k_chain<LDSA, RING, EPI, NJ, KB><<<256, 256>>>(w, out, ticks, iters);
  k_chain<LDSA, RING, EPI, NJ, KB><<<256, 256>>>(w, out, ticks, iters);
  hipDeviceSynchronize();
  unsigned long long h[1024];
  hipMemcpy(h, ticks, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 1024; ++i) avg += h[i];
  avg /= 1024;
  const double mf = (double)iters * KB * 4 * NJ * 2;
  printf("%-34s ticks/chain=%.0f  ticks/MFMA=%.1f (ideal 32)\n", name, avg / iters, avg / mf);
}

int main() {
  float4* w;
  float* out;
  unsigned long long* ticks;
  hipMalloc(&w, sizeof(float4) * 8 * 64 * 64 * 64 + 4096);
  hipMemset(w, 0, sizeof(float4) * 8 * 64 * 64 * 64);
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&ticks, 1024 * 8);
  run<false, false, false, 4, 4>("regs only", w, out, ticks);
  run<true, false, false, 4, 4>("lds A", w, out, ticks);
  run<false, true, false, 4, 4>("ring B", w, out, ticks);
  run<false, false, true, 4, 4>("epilogue", w, out, ticks);
  run<true, true, false, 4, 4>("lds A + ring B", w, out, ticks);
  run<true, true, true, 4, 4>("lds A + ring B + epilogue", w, out, ticks);
  run<true, true, true, 1, 16>("NJ1 KB16 all", w, out, ticks);
  run<false, false, false, 1, 16>("NJ1 KB16 regs only", w, out, ticks);
  return 0;
}
