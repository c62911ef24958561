// Microbenchmark (diagnostic, not shipped): the memory ceilings of the search's select / backup at the
// footprints and concurrency the wave kernel runs them (mzh_wave_kernel<2>: 2,048 waves = two per SIMD,
// 32 roots per wave, a lane pair per root, each lane loading its half of a 128-B tree block per level).
//   chase : every root walks a random cycle of 128-B blocks, the next block index from the loaded line
//           (a selection level's dependent block load): ns per level = the LOADED latency at that footprint
//   stream: the same loads without the dependency (each root's next block from a hash): the random-line
//           bandwidth ceiling (GB/s of whole 128-B lines) at that footprint
// Footprints: 16 MB (L2-resident), 128 MB (Infinity Cache), 448 MB (configs[2]'s tree blocks on one GPU:
// 65,536 roots x 51 blocks x 128 B = 428 MB), 1.3 GB (blocks + the fused kernel's latents).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/tree_mem_probe.hip -o tools/micro/tree_mem_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

constexpr int WG = 512, THREADS = 256;  // 2,048 waves: two per SIMD, like the wave kernel at 65,536 roots

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// word 0 of every block holds the next block of a random cyclic permutation of all blocks
// pairs: roots per wave that walk (32 = the wave kernel's load; fewer = the same waves, lighter traffic)
template <bool CHASE>
__global__ __launch_bounds__(THREADS, 2) void walk(const uint4* __restrict__ buf, uint32_t nblk, int levels,
                                                   uint32_t* out, int pairs) {
  const int lane = threadIdx.x & 63;
  const uint32_t root = (blockIdx.x * THREADS + threadIdx.x) >> 1;  // a lane pair per root
  uint32_t idx = mix(root * 2654435761u) % nblk;
  uint32_t acc = 0;
  if ((lane >> 1) >= pairs) levels = 0;
#pragma unroll 4
  for (int l = 0; l < levels; ++l) {
    const uint4* b = buf + (size_t)idx * 8 + (lane & 1) * 4;  // this lane's half block: 4 x 16 B
    const uint4 v0 = b[0], v1 = b[1], v2 = b[2], v3 = b[3];
    acc += v1.x + v2.y + v3.z;
    if (CHASE) {
      // the pair's next block: lane 0's word 0, given to its partner (the group take of a selection level)
      const uint32_t nx = __shfl_xor((int)v0.x, 1);
      idx = (lane & 1) ? nx : v0.x;
    } else {
      idx = mix(idx + root + (uint32_t)l * 40503u + (v0.x & 0)) % nblk;
    }
  }
  out[blockIdx.x * THREADS + threadIdx.x] = acc + idx;
}

int main() {
  const size_t foot_mb[] = {16, 128, 448, 1344};
  uint32_t* out;
  CHECK(hipMalloc(&out, (size_t)WG * THREADS * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("[\n");
  for (size_t fi = 0; fi < sizeof(foot_mb) / sizeof(foot_mb[0]); ++fi) {
    const uint32_t nblk = (uint32_t)(foot_mb[fi] * 1024 * 1024 / 128);
    std::vector<uint32_t> next(nblk), perm(nblk);
    for (uint32_t i = 0; i < nblk; ++i) perm[i] = i;
    uint64_t s = 88172645463325252ull;
    for (uint32_t i = nblk - 1; i > 0; --i) {  // Fisher-Yates: one random cycle through every block
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      const uint32_t j = (uint32_t)(s % (i + 1));
      const uint32_t t = perm[i];
      perm[i] = perm[j];
      perm[j] = t;
    }
    for (uint32_t i = 0; i < nblk; ++i) next[perm[i]] = perm[(i + 1) % nblk];
    std::vector<uint32_t> host((size_t)nblk * 32, 0);
    for (uint32_t i = 0; i < nblk; ++i) host[(size_t)i * 32] = next[i];
    uint4* buf;
    CHECK(hipMalloc(&buf, host.size() * 4));
    CHECK(hipMemcpy(buf, host.data(), host.size() * 4, hipMemcpyHostToDevice));
    const int levels = 400;
    const int pair_set[] = {32, 8, 1};
    for (int pi = 0; pi < 3; ++pi) {
      const int pairs = pair_set[pi];
      float ms[2] = {0, 0};
      for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {  // the last of three launches is timed (first ones warm the caches)
          CHECK(hipEventRecord(e0, 0));
          if (mode == 0)
            hipLaunchKernelGGL(walk<true>, dim3(WG), dim3(THREADS), 0, 0, buf, nblk, levels, out, pairs);
          else
            hipLaunchKernelGGL(walk<false>, dim3(WG), dim3(THREADS), 0, 0, buf, nblk, levels, out, pairs);
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms[mode], e0, e1));
        }
      }
      const double roots = (double)WG * (THREADS / 64) * pairs;
      const double lines = roots * levels;
      printf("  {\"footprint_mb\": %zu, \"roots_walking\": %.0f, \"roots_per_wave\": %d, \"levels\": %d, "
             "\"chase_ms\": %.4f, \"chase_ns_per_level\": %.1f, \"chase_line_gbps\": %.1f, \"stream_ms\": %.4f, "
             "\"stream_line_gbps\": %.1f}%s\n",
             foot_mb[fi], roots, pairs, levels, ms[0], ms[0] * 1e6 / levels, lines * 128 / (ms[0] * 1e-3) / 1e9, ms[1],
             lines * 128 / (ms[1] * 1e-3) / 1e9,
             (fi + 1 < sizeof(foot_mb) / sizeof(foot_mb[0]) || pi < 2) ? "," : "");
    }
    CHECK(hipFree(buf));
  }
  printf("]\n");
  return 0;
}
