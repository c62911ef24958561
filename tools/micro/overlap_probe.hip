// Microbenchmark (diagnostic, not shipped): can a latency-bound tree walk -- dependent 128-B block
// loads from L2, each followed by a dependent fp64 chain and a DPP argmax -- hide under a stream of
// v_mfma_f32_16x16x4_f32 on the same SIMD?  One workgroup per CU (256 CUs); per level: one block load
// per 8-lane group, VPL dependent fp64 FMAs, three DPP max steps, the next block index from the load
// and the chain; MPL MFMAs per level on 4 independent accumulators, operands in registers.
//   mode 0  MFMA stream alone           (4 waves, one per SIMD)
//   mode 1  tree walk alone             (4 waves)
//   mode 2  both in ONE wave's instruction stream, interleaved by the scheduler (sched_group_barrier:
//           the load issued first, MPL/2 MFMAs under its latency, then 1 MFMA : 1 VALU)
//   mode 3  both on one SIMD in TWO waves (8 waves: waves 0-3 MFMA, 4-7 tree), the hardware interleaves
//   mode 4  as mode 2 but the tree part is the wave's own instruction order (no interleave hints)
// Prints ticks per level per wave (s_memtime) for each mode: overlap is good if mode 2 / 3 approach
// max(mode 0, mode 1) rather than mode 0 + mode 1.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int NBLK = 512;  // blocks of 128 B per workgroup region: 64 KB, L2-resident

__device__ __forceinline__ float dpp_max8(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true)));
  return v;
}

// one 32-cycle unit of matrix work: one v_mfma_f32_16x16x4_f32 (K4 = 0), or four v_mfma_f32_4x4x1_16b_f32
// (K4 = 1: the same 1,024 MACs and pipe time in 8-cycle instructions, so a co-resident wave's VALU waits
// at most one short MFMA instead of a 32-cycle one)
template <int K4>
__device__ __forceinline__ floatx4 mf(float a, float b, floatx4 c) {
  if (K4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b + (float)i, c, 0, 0, 0);
    return c;
  }
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int MODE, int MPL, int VPL, int K4 = 0>
__global__ __launch_bounds__(512, 1) void k(const uint4* chase, float* out, unsigned long long* ticks, int levels) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* reg = chase + (size_t)blockIdx.x * NBLK * 8;
  // modes 5 / 6: mode 3 with the tree waves / the MFMA waves at s_setprio 3 (the other at 0)
  const bool pair = MODE == 3 || MODE == 5 || MODE == 6;
  const bool do_mfma = MODE == 0 || MODE == 2 || MODE == 4 || (pair && wave < 4);
  const bool do_tree = MODE == 1 || MODE == 2 || MODE == 4 || (pair && wave >= 4);
  if ((MODE == 5 && wave >= 4) || (MODE == 6 && wave < 4)) __builtin_amdgcn_s_setprio(3);
  floatx4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a[8], b[8];  // distinct operands per MFMA (as the MLP's weight fragments / activations)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = 1e-3f * (lane + j);
    b[j] = 2e-3f * (lane + wave + j);
  }
  uint32_t idx = (lane >> 3) * 7 + wave * 61;
  double x = 1.0 + 1e-3 * lane;
  const double c1 = 0.99999, c2 = 1e-7;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < levels; ++l) {
    if (do_tree && do_mfma) {
      const uint4 v = reg[(idx % NBLK) * 8 + (lane & 7)];
#pragma unroll
      for (int q = 0; q < MPL / 2; ++q) acc[q & 3] = mf<K4>(a[q & 7], b[q & 7], acc[q & 3]);
      x = x + (double)v.y * 1e-9;
#pragma unroll
      for (int q = 0; q < VPL; ++q) x = __builtin_fma(x, c1, c2);
      const float m = dpp_max8((float)x + (float)(lane & 7));
      idx = v.x + (m > 1e30f ? 1u : 0u);
#pragma unroll
      for (int q = MPL / 2; q < MPL; ++q) acc[q & 3] = mf<K4>(a[q & 7], b[q & 7], acc[q & 3]);
      if (MODE == 2) {
        // the load, MPL/2 MFMAs under it, then the chain interleaved 1 MFMA : 1 VALU
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // the load's address
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MPL / 2, 0);
#pragma unroll
        for (int q = 0; q < MPL / 2; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
      }
    } else if (do_tree) {
      const uint4 v = reg[(idx % NBLK) * 8 + (lane & 7)];
      x = x + (double)v.y * 1e-9;
#pragma unroll
      for (int q = 0; q < VPL; ++q) x = __builtin_fma(x, c1, c2);
      const float m = dpp_max8((float)x + (float)(lane & 7));
      idx = v.x + (m > 1e30f ? 1u : 0u);
    } else if (do_mfma) {
#pragma unroll
      for (int q = 0; q < MPL; ++q) acc[q & 3] = mf<K4>(a[q & 7], b[q & 7], acc[q & 3]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = (float)x + (float)idx;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) ticks[blockIdx.x * 8 + wave] = t1 - t0;
}

// dependent 128-B block loads alone (one 8-lane group per block, 16 B per lane, the next index from the
// loaded word): the L2 / MALL latency of one selection level's block wait, per footprint
__global__ __launch_bounds__(256, 1) void chase_lat(const uint4* chase, float* out, unsigned long long* ticks, int levels,
                                                    int nblk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* reg = chase + (size_t)blockIdx.x * nblk * 8;
  uint32_t idx = (lane >> 3) * 7 + wave * 61;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < levels; ++l) idx = reg[(idx % nblk) * 8 + (lane & 7)].x;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)idx;
  if (lane == 0) ticks[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int MODE, int MPL, int VPL, int K4 = 0>
static double run(const uint4* chase, float* out, unsigned long long* ticks, int levels) {
  const int threads = (MODE == 3 || MODE == 5 || MODE == 6) ? 512 : 256;
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k<MODE, MPL, VPL, K4>), dim3(256), dim3(threads), 0, 0, chase, out, ticks, levels);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(256 * 8);
  hipMemcpy(h.data(), ticks, h.size() * 8, hipMemcpyDeviceToHost);
  // per workgroup: the slowest wave
  double avg = 0;
  for (int b = 0; b < 256; ++b) {
    unsigned long long m = 0;
    for (int w = 0; w < threads / 64; ++w) m = h[b * 8 + w] > m ? h[b * 8 + w] : m;
    avg += (double)m;
  }
  return avg / 256 / levels;
}

template <int MPL, int VPL>
static void sweep(const uint4* chase, float* out, unsigned long long* ticks) {
  const int L = 2000;
  const double m0 = run<0, MPL, VPL>(chase, out, ticks, L), m1 = run<1, MPL, VPL>(chase, out, ticks, L);
  const double m2 = run<2, MPL, VPL>(chase, out, ticks, L), m3 = run<3, MPL, VPL>(chase, out, ticks, L);
  const double m4 = run<4, MPL, VPL>(chase, out, ticks, L);
  printf("{\"mfma_per_level\": %d, \"fp64_chain_per_level\": %d, \"ticks_per_level\": {\"mfma_alone\": %.1f, "
         "\"tree_alone\": %.1f, \"one_wave_interleaved\": %.1f, \"two_waves_per_simd\": %.1f, "
         "\"one_wave_unhinted\": %.1f}, \"sum\": %.1f, \"max\": %.1f}\n",
         MPL, VPL, m0, m1, m2, m3, m4, m0 + m1, m0 > m1 ? m0 : m1);
}

// per workgroup region: a random cyclic permutation of its nblk blocks (word 0 of each lane's 16 B =
// the next block)
static std::vector<uint32_t> make_chase(int nblk) {
  std::vector<uint32_t> host((size_t)256 * nblk * 32);
  uint64_t s = 12345;
  std::vector<uint32_t> perm(nblk);
  for (int b = 0; b < 256; ++b) {
    for (int i = 0; i < nblk; ++i) perm[i] = i;
    for (int i = nblk - 1; i > 0; --i) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      const int j = (int)((s >> 33) % (uint64_t)(i + 1));
      const uint32_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
    for (int i = 0; i < nblk; ++i)
      for (int w = 0; w < 32; ++w) host[((size_t)b * nblk + perm[i]) * 32 + w] = (w % 4 == 0) ? perm[(i + 1) % nblk] : 1000u + w;
  }
  return host;
}

// the same two-waves-per-SIMD pairing with the matrix work as 8-cycle 4x4x1 MFMAs
template <int MPL, int VPL>
static void sweep_k4(const uint4* chase, float* out, unsigned long long* ticks) {
  const int L = 2000;
  const double m0 = run<0, MPL, VPL, 1>(chase, out, ticks, L), m1 = run<1, MPL, VPL, 1>(chase, out, ticks, L);
  const double m3 = run<3, MPL, VPL, 1>(chase, out, ticks, L);
  const double m5 = run<5, MPL, VPL, 1>(chase, out, ticks, L), m6 = run<6, MPL, VPL, 1>(chase, out, ticks, L);
  const double p5 = run<5, MPL, VPL, 0>(chase, out, ticks, L), p6 = run<6, MPL, VPL, 0>(chase, out, ticks, L);
  printf("{\"mfma_4x4x1_units_per_level\": %d, \"fp64_chain_per_level\": %d, \"ticks_per_level\": {\"mfma_alone\": %.1f, "
         "\"tree_alone\": %.1f, \"two_waves_per_simd\": %.1f, \"two_waves_tree_prio\": %.1f, \"two_waves_mfma_prio\": %.1f, "
         "\"16x16x4_two_waves_tree_prio\": %.1f, \"16x16x4_two_waves_mfma_prio\": %.1f}, \"sum\": %.1f, \"max\": %.1f}\n",
         MPL, VPL, m0, m1, m3, m5, m6, p5, p6, m0 + m1, m0 > m1 ? m0 : m1);
}

int main() {
  float* out;
  unsigned long long* ticks;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&ticks, 256 * 8 * 8);
  for (int nblk : {512, 4096, 32768}) {  // 64 KB, 512 KB, 4 MB per workgroup = 16 MB, 128 MB, 1 GB in all
    std::vector<uint32_t> host = make_chase(nblk);
    uint4* c;
    hipMalloc(&c, host.size() * 4);
    hipMemcpy(c, host.data(), host.size() * 4, hipMemcpyHostToDevice);
    const int L = 4000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(chase_lat, dim3(256), dim3(256), 0, 0, c, out, ticks, L, nblk);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(chase_lat, dim3(256), dim3(256), 0, 0, c, out, ticks, L, nblk);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(256 * 8);
    hipMemcpy(h.data(), ticks, h.size() * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < 256; ++b)
      for (int w = 0; w < 4; ++w) avg += (double)h[b * 8 + w];
    // s_memtime ticks per ns from the same launch (the slowest wave's ticks over the event time)
    unsigned long long mx = 0;
    for (int b = 0; b < 256; ++b)
      for (int w = 0; w < 4; ++w) mx = h[b * 8 + w] > mx ? h[b * 8 + w] : mx;
    printf("{\"chase_footprint_mb\": %.1f, \"ticks_per_dependent_block_load\": %.1f, \"ns_per_load\": %.1f, "
           "\"memtime_ticks_per_ns\": %.3f}\n", 256.0 * nblk * 128 / 1048576.0, avg / 1024 / L, ms * 1e6 / L,
           (double)mx / (ms * 1e6));
    hipFree(c);
  }
  std::vector<uint32_t> host = make_chase(NBLK);
  uint4* chase;
  hipMalloc(&chase, host.size() * 4);
  hipMemcpy(chase, host.data(), host.size() * 4, hipMemcpyHostToDevice);
  sweep<16, 8>(chase, out, ticks);
  sweep<32, 16>(chase, out, ticks);
  sweep<48, 24>(chase, out, ticks);
  sweep<48, 48>(chase, out, ticks);
  sweep<96, 24>(chase, out, ticks);
  sweep_k4<16, 8>(chase, out, ticks);
  sweep_k4<32, 16>(chase, out, ticks);
  sweep_k4<48, 24>(chase, out, ticks);
  sweep_k4<96, 24>(chase, out, ticks);
  return 0;
}
