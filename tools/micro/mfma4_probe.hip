// Microbenchmark (diagnostic, not shipped): can a 16-row tile's single K = 256 accumulation chain run
// at the matrix pipe's rate as v_mfma_f32_4x4x1_16b_f32 steps instead of dependent
// v_mfma_f32_16x16x4_f32 ones (whose 40-tick dependent latency exceeds their 32-tick issue)?
//   1. layout: the 4x4x1_16b operand / result lanes, decoded from an outer product
//   2. rate: one wave per SIMD, a single dependent chain (and two interleaved chains) of each form
//   3. numerics: a 16 x 16 x 256 tile as a 4x4x1 chain (k = 0..255) against the 16x16x4 chain
//      (k-blocks of 4 consecutive k) -- bit for bit, and both against a host fmaf chain
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(float* out) {
  const int l = threadIdx.x;
  // A operand of lane l: l + 1 (< 256); B operand: 2^(8 (l % 4)) -- each product a * b decodes uniquely
  const float a = (float)(l + 1), b = (float)(1u << (8 * (l & 3)));
  floatx4 c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, floatx4{0, 0, 0, 0}, 0, 0, 0);
  for (int v = 0; v < 4; ++v) out[l * 4 + v] = c[v];
}

// single dependent chain (CH = 1) or CH interleaved chains, N steps per chain
template <int FORM, int CH>
__global__ __launch_bounds__(256, 1) void k_rate(float* out, unsigned long long* ticks, int n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  floatx4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = floatx4{0, 0, 0, 0};
  float a[8], b[8];
  for (int j = 0; j < 8; ++j) {
    a[j] = 1e-3f * (lane + j);
    b[j] = 2e-3f * (lane - j);
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int c = 0; c < CH; ++c)
        acc[c] = FORM ? __builtin_amdgcn_mfma_f32_4x4x1f32(a[j], b[j], acc[c], 0, 0, 0)
                      : __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc[c], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) ticks[blockIdx.x * 4 + wave] = t1 - t0;
}

// numerics: A [16][256], B [256][16] (row-major), C = A.B as (a) 16x16x4 chain, (b) 4x4x1 chain
// layouts (from k_layout, checked on the host): 16x16x4 A lane (r, g) = A[r][4s+g], B lane (c, g) = B[4s+g][c],
// D lane (c, g) reg i = C[4g+i][c]; 4x4x1_16b: block q = lane / 4 ... decoded at run time (lay[])
__global__ void k_num(const float* A, const float* B, float* C16, float* C4, const int* lay) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  floatx4 acc = {0, 0, 0, 0};
  for (int s = 0; s < 64; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[r * 256 + 4 * s + g], B[(4 * s + g) * 16 + r], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C16[(4 * g + i) * 16 + r] = acc[i];
  // 4x4x1: lay[l * 3 + {0,1,2}] = (block, A-row index, B-col index) of lane l's operands; the 16 blocks
  // tile the 16x16 output as block q -> rows 4(q / 4).., cols 4(q % 4)..
  const int q = lay[l * 3], ai = lay[l * 3 + 1], bj = lay[l * 3 + 2];
  const int row = 4 * (q >> 2) + ai, col = 4 * (q & 3) + bj;
  floatx4 d = {0, 0, 0, 0};
  for (int k = 0; k < 256; ++k) d = __builtin_amdgcn_mfma_f32_4x4x1f32(A[row * 256 + k], B[k * 16 + col], d, 0, 0, 0);
  for (int v = 0; v < 4; ++v) {
    const int o = lay[192 + l * 8 + 2 * v], p = lay[192 + l * 8 + 2 * v + 1];  // result (row, col) in block
    C4[(4 * (q >> 2) + o) * 16 + 4 * (q & 3) + p] = d[v];
  }
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, d);
  std::vector<float> h(256);
  hipMemcpy(h.data(), d, 256 * 4, hipMemcpyDeviceToHost);
  // decode: value = (la + 1) * 2^(8 jb): la = the lane whose A operand entered, jb = the B lane's index % 4
  std::vector<int> lay(192 + 64 * 8);
  bool ok = true;
  printf("{\"layout\": [");
  for (int l = 0; l < 64; ++l) {
    for (int v = 0; v < 4; ++v) {
      const float val = h[l * 4 + v];
      int jb = 0;
      while (jb < 3 && val >= 256.0f * (float)(1u << (8 * jb))) ++jb;
      const float av = val / (float)(1u << (8 * jb));
      const int la = (int)av - 1;
      if (av != (float)(la + 1) || la < 0 || la > 63 || la / 4 != l / 4) ok = false;
      lay[192 + l * 8 + 2 * v] = la % 4;      // result row within the block = the A lane's index
      lay[192 + l * 8 + 2 * v + 1] = jb;      // result col within the block = the B lane's index
      if (l < 8) printf("%s[%d,%d,%d,%d]", (l || v) ? "," : "", l, v, la, jb);
    }
    lay[l * 3] = l / 4;  // lane l supplies A row l % 4 and B col l % 4 of block l / 4 (checked by `decoded`)
    lay[l * 3 + 1] = l % 4;
    lay[l * 3 + 2] = l % 4;
  }
  printf("], \"decoded\": %s}\n", ok ? "true" : "false");
  // rate
  float* out;
  unsigned long long* ticks;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&ticks, 256 * 4 * 8);
  auto rate = [&](auto kern, const char* name) {
    const int n = 4096;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, out, ticks, n);
    hipDeviceSynchronize();
    std::vector<unsigned long long> t(1024);
    hipMemcpy(t.data(), ticks, 1024 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto x : t) s += (double)x;
    printf("{\"chain\": \"%s\", \"ticks_per_instruction\": %.2f}\n", name, s / 1024 / n);
  };
  rate(k_rate<0, 1>, "16x16x4 x1");
  rate(k_rate<0, 2>, "16x16x4 x2 (per instruction of one chain)");
  rate(k_rate<1, 1>, "4x4x1_16b x1");
  rate(k_rate<1, 2>, "4x4x1_16b x2 (per instruction of one chain)");
  rate(k_rate<1, 4>, "4x4x1_16b x4 (per instruction of one chain)");
  // numerics
  std::vector<float> A(16 * 256), B(256 * 16);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
  for (auto& x : A) x = rnd();
  for (auto& x : B) x = rnd() * 0.37f;
  float *dA, *dB, *d16, *d4;
  int* dl;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dB, B.size() * 4);
  hipMalloc(&d16, 256 * 4);
  hipMalloc(&d4, 256 * 4);
  hipMalloc(&dl, lay.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dl, lay.data(), lay.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_num, dim3(1), dim3(64), 0, 0, dA, dB, d16, d4, dl);
  std::vector<float> c16(256), c4(256);
  hipMemcpy(c16.data(), d16, 1024, hipMemcpyDeviceToHost);
  hipMemcpy(c4.data(), d4, 1024, hipMemcpyDeviceToHost);
  int eq164 = 0, eq16h = 0, eq4h = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float acc = 0.0f;
      for (int k = 0; k < 256; ++k) acc = fmaf(A[i * 256 + k], B[k * 16 + j], acc);
      eq164 += c16[i * 16 + j] == c4[i * 16 + j];
      eq16h += c16[i * 16 + j] == acc;
      eq4h += c4[i * 16 + j] == acc;
    }
  printf("{\"numerics\": {\"16x16x4_eq_4x4x1\": %d, \"16x16x4_eq_host_fmaf\": %d, \"4x4x1_eq_host_fmaf\": %d, \"of\": 256}}\n",
         eq164, eq16h, eq4h);
  return 0;
}
