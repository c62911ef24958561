// Microbenchmark: does independent VALU work issued between v_mfma_f32_16x16x4_f32 instructions of
// the same wave hide under the MFMA's 32-cycle issue interval (one wave per SIMD)?  NV VALU ops
// (dependent pairs on 4 independent chains) per MFMA; 8 accumulators.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NV, bool F64>
__global__ __launch_bounds__(256, 1) void k(float* out, unsigned long long* ticks, int iters) {
  const int lane = threadIdx.x & 63;
  floatx4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a = 1e-3f * lane, b = 2e-3f * lane;
  float v[4] = {1.f + lane, 2.f, 3.f, 4.f};
  double d[4] = {1.0 + lane, 2.0, 3.0, 4.0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        if (F64) d[q & 3] = d[q & 3] * 1.0000001 + 1e-9;
        else v[q & 3] = v[q & 3] * 1.0000001f + 1e-9f;
      }
    }
    a += 1e-7f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0];
  s += v[0] + v[1] + v[2] + v[3] + (float)(d[0] + d[1] + d[2] + d[3]);
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) ticks[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int NV, bool F64>
void run(float* out, unsigned long long* ticks) {
  const int iters = 2000;
  k<NV, F64><<<256, 256>>>(out, ticks, iters);
  k<NV, F64><<<256, 256>>>(out, ticks, iters);
  hipDeviceSynchronize();
  unsigned long long h[1024];
  hipMemcpy(h, ticks, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 1024; ++i) avg += h[i];
  avg /= 1024;
  printf("%s VALU ops per MFMA=%2d  ticks/MFMA=%.1f\n", F64 ? "f64" : "f32", NV, avg / (iters * 8.0));
}

int main() {
  float* out;
  unsigned long long* ticks;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&ticks, 1024 * 8);
  run<0, false>(out, ticks);
  run<2, false>(out, ticks);
  run<4, false>(out, ticks);
  run<6, false>(out, ticks);
  run<8, false>(out, ticks);
  run<12, false>(out, ticks);
  run<2, true>(out, ticks);
  run<4, true>(out, ticks);
  return 0;
}
