// Microbenchmark: v_mfma_f32_16x16x4_f32 issue rate per SIMD for one vs two waves per SIMD,
// NACC independent accumulators, with / without LDS-fed A operands (diagnostic only, not shipped).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NACC, int LDSA>
__global__ void k_mfma(float* out, unsigned long long* ticks, int iters) {
  __shared__ float lds[4096];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 1e-3f * (i & 7);
  __syncthreads();
  floatx4 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a = 1e-3f * lane, b = 2e-3f * lane;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (LDSA) {
      float av[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) av[q] = lds[(lane + 64 * q + 256 * (it & 7)) & 4095];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], b, acc[j], 0, 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) ticks[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int NACC, int LDSA>
void run(const char* name, int waves_per_cu, int iters) {
  const int blocks = 256, threads = 64 * waves_per_cu;
  float* out;
  unsigned long long* ticks;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&ticks, blocks * waves_per_cu * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_mfma<NACC, LDSA><<<blocks, threads>>>(out, ticks, iters);
  hipEventRecord(e0);
  k_mfma<NACC, LDSA><<<blocks, threads>>>(out, ticks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = new unsigned long long[blocks * waves_per_cu];
  hipMemcpy(h, ticks, blocks * waves_per_cu * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks * waves_per_cu; ++i) avg += h[i];
  avg /= blocks * waves_per_cu;
  const double mfma_per_wave = (double)iters * 4 * NACC;
  const double per_simd = mfma_per_wave * waves_per_cu / 4;
  printf("%-28s waves/CU=%d  ticks/MFMA(wave)=%.1f  ticks/MFMA(SIMD)=%.1f  ms=%.3f  TFLOP/s=%.1f\n", name,
         waves_per_cu, avg / mfma_per_wave, avg / per_simd, ms, per_simd * 4 * 256 * 2048.0 / (ms * 1e-3) / 1e12);
  delete[] h;
  hipFree(out);
  hipFree(ticks);
}

int main() {
  const int it = 4096;
  run<8, 0>("nacc8", 4, it);
  run<8, 0>("nacc8", 8, it);
  run<4, 0>("nacc4", 4, it);
  run<2, 0>("nacc2", 4, it);
  run<2, 0>("nacc2", 8, it);
  run<1, 0>("nacc1", 4, it);
  run<8, 1>("nacc8 lds-A", 4, it);
  run<2, 1>("nacc2 lds-A", 4, it);
  run<8, 1>("nacc8 lds-A", 8, it);
  return 0;
}
