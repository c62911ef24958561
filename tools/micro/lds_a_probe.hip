// Microbenchmark: where the LDS-fed A operand of the search MLP's MFMA chunk (NJ=4 tiles x MT=2 row
// tiles x KB=4 k-blocks = 128 v_mfma_f32_16x16x4_f32 per wave) costs issue rate.  Variants:
//   DIST  A reads issued DIST k-blocks ahead (1 = the shipped double buffer, 2 = triple buffer)
//   SB    a sched_barrier at every k-block boundary (shipped) or none
//   XPF   the next chunk's k-block-0 A reads issued during this chunk's last k-block (else they are
//         issued at the chunk start and waited for)
// One wave per SIMD, 256 workgroups.  Diagnostic only, not shipped.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int DIST, bool SB, bool XPF>
__global__ __launch_bounds__(256, 1) void k_probe(float* out, unsigned long long* ticks, int iters) {
  constexpr int NJ = 4, KB = 4, NB = DIST + 1;
  __shared__ __attribute__((aligned(16))) float lds[32 * 68 * 2];
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < 32 * 68 * 2; i += 256) lds[i] = 1e-3f * (i & 15);
  __syncthreads();
  floatx4 f[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) f[s] = floatx4{1e-3f * s, 2e-3f, 3e-3f, 1e-3f * lane};
  const float* arow0 = lds + r * 68 + 4 * g;
  floatx4 keep = {0, 0, 0, 0};
  floatx4 a[NB][2];
  // k-block k of chunk `it` reads buffer (it & 1) (two alternating A images), columns 16k..16k+15
  auto aptr = [&](int it, int kb, int m) { return arow0 + (it & 1) * 32 * 68 + m * 16 * 68 + kb * 16; };
  if (XPF) {
#pragma unroll
    for (int d = 0; d < DIST; ++d)
#pragma unroll
      for (int m = 0; m < 2; ++m) a[d % NB][m] = *reinterpret_cast<const floatx4*>(aptr(0, d, m));
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    floatx4 acc[NJ][2];
    if (!XPF) {
#pragma unroll
      for (int d = 0; d < DIST; ++d)
#pragma unroll
        for (int m = 0; m < 2; ++m) a[d % NB][m] = *reinterpret_cast<const floatx4*>(aptr(it, d, m));
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      // the read DIST k-blocks ahead: this chunk's, or (XPF) the next chunk's first ones
      const int kn = kb + DIST;
      if (kn < KB) {
#pragma unroll
        for (int m = 0; m < 2; ++m) a[kn % NB][m] = *reinterpret_cast<const floatx4*>(aptr(it, kn, m));
      } else if (XPF) {
#pragma unroll
        for (int m = 0; m < 2; ++m) a[kn % NB][m] = *reinterpret_cast<const floatx4*>(aptr(it + 1, kn - KB, m));
      }
      if (SB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < NJ; ++q)
#pragma unroll
          for (int m = 0; m < 2; ++m)
            acc[q][m] = j == 0 && kb == 0
                            ? __builtin_amdgcn_mfma_f32_16x16x4f32(a[kb % NB][m][j], f[q * KB + kb][j], floatx4{0, 0, 0, 0}, 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x4f32(a[kb % NB][m][j], f[q * KB + kb][j], acc[q][m], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NJ; ++q) keep += acc[q][0] + acc[q][1];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = keep[0] + keep[1] + keep[2] + keep[3];
  if (lane == 0) ticks[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

// register-only operands: MODE 1 = distinct A per (m, j), B per tile; 2 = distinct A and B per MFMA;
// 4..6 = as 2 with B taken from tuple position (j + MODE - 3) & 3 (another VGPR bank than A's).
// (Modes 0 / 3 -- one A or one B register for every MFMA -- make whole accumulator chains identical,
// which the compiler merges: they time fewer MFMAs than they count and are not run.)
template <int MODE, int WPS = 1>
__global__ __launch_bounds__(256, WPS) void k_regs(float* out, unsigned long long* ticks, int iters) {
  constexpr int NJ = 4, KB = 4;
  const int lane = threadIdx.x & 63;
  floatx4 f[16];
#pragma unroll
  for (int s = 0; s < 16; ++s)
    f[s] = floatx4{1e-3f * (s + lane), 2e-3f * (s + 2 * lane), 3e-3f * (s + 3 * lane), 4e-3f * (s + 5 * lane)};
  floatx4 a[2];
  a[0] = floatx4{1e-3f * lane, 2e-3f * lane, 3e-3f * lane, 4e-3f * lane};
  a[1] = floatx4{5e-3f * lane, 6e-3f * lane, 7e-3f * lane, 8e-3f * lane};
  floatx4 keep = {0, 0, 0, 0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    floatx4 acc[NJ][2];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < NJ; ++q)
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            const float av = MODE == 0 ? a[0][0] : a[m][j];
            const float bv = MODE == 3   ? f[0][0]
                             : MODE == 2 ? f[q * KB + kb][j]
                             : MODE >= 4 ? f[q * KB + kb][(j + MODE - 3) & 3]
                                         : f[q * KB][0];
            acc[q][m] = (j == 0 && kb == 0) ? __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, floatx4{0, 0, 0, 0}, 0, 0, 0)
                                            : __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[q][m], 0, 0, 0);
          }
#pragma unroll
    for (int q = 0; q < NJ; ++q) keep += acc[q][0] + acc[q][1];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = keep[0] + keep[1] + keep[2] + keep[3];
  if (lane == 0) ticks[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE, int WPS = 1>
void run_regs(const char* name, float* out, unsigned long long* ticks) {
  const int iters = 20000 / WPS;
  k_regs<MODE, WPS><<<256 * WPS, 256>>>(out, ticks, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  k_regs<MODE, WPS><<<256 * WPS, 256>>>(out, ticks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  // one workgroup per CU, one wave per SIMD: 256 x 4 waves x iters x 128 MFMAs x 1024 MAC x 2
  printf("%-40s wall %.3f ms = %.1f TFLOP/s fp32 MFMA\n", name, ms, 256.0 * WPS * 4 * iters * 128 * 2048 / (ms * 1e-3) / 1e12);
  unsigned long long h[1024];
  hipMemcpy(h, ticks, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 1024; ++i) avg += h[i];
  avg /= 1024;
  printf("%-40s ticks/MFMA=%.2f (ideal 32)\n", name, avg / ((double)iters * 128));
}

template <int DIST, bool SB, bool XPF>
void run(const char* name, float* out, unsigned long long* ticks) {
  const int iters = 2000;
  k_probe<DIST, SB, XPF><<<256, 256>>>(out, ticks, iters);
  k_probe<DIST, SB, XPF><<<256, 256>>>(out, ticks, iters);
  hipDeviceSynchronize();
  unsigned long long h[1024];
  hipMemcpy(h, ticks, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 1024; ++i) avg += h[i];
  avg /= 1024;
  printf("%-40s ticks/MFMA=%.2f (ideal 32)\n", name, avg / ((double)iters * 128));
}

int main() {
  float* out;
  unsigned long long* ticks;
  hipMalloc(&out, 512 * 256 * 4);
  hipMalloc(&ticks, 2048 * 8);
  run_regs<1>("regs: A per (m,j), B per tile", out, ticks);
  run_regs<2>("regs: A per (m,j), B per (tile,kb,j)", out, ticks);
  run_regs<2, 2>("regs: as 2, two waves per SIMD", out, ticks);
  run_regs<4>("regs: as 2, B position j+1", out, ticks);
  run_regs<5>("regs: as 2, B position j+2", out, ticks);
  run_regs<6>("regs: as 2, B position j+3", out, ticks);
  run<1, true, false>("dist1 sb (shipped)", out, ticks);
  run<1, false, false>("dist1 no-sb", out, ticks);
  run<1, true, true>("dist1 sb + next-chunk prefetch", out, ticks);
  run<2, true, false>("dist2 sb", out, ticks);
  run<2, true, true>("dist2 sb + next-chunk prefetch", out, ticks);
  run<2, false, true>("dist2 no-sb + next-chunk prefetch", out, ticks);
  return 0;
}
