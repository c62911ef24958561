// Dependent fp32 FMA chain cost on gfx950, one wave alone on its SIMD (the latency kernel's K = 256 chains,
// csrc/mzh_one.hip): cycles per step of 1024 dependent v_fmac_f32 (a) with both operands in VGPRs, (b) with
// the multiplicand broadcast by DPP row_newbcast, (c) two independent chains interleaved, (d) four.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/fmac_chain_probe.hip -o tools/micro/fmac_chain_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define F1 "v_fmac_f32 %0, %1, %2\n\t"
#define D1(j) "v_fmac_f32_dpp %0, %1, %2 row_newbcast:" #j " row_mask:0xf bank_mask:0xf\n\t"
#define F16 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1 F1
#define D16 D1(0) D1(1) D1(2) D1(3) D1(4) D1(5) D1(6) D1(7) D1(8) D1(9) D1(10) D1(11) D1(12) D1(13) D1(14) D1(15)
#define F2 "v_fmac_f32 %0, %2, %3\n\tv_fmac_f32 %1, %2, %3\n\t"
#define F2x8 F2 F2 F2 F2 F2 F2 F2 F2
#define F4 "v_fmac_f32 %0, %4, %5\n\tv_fmac_f32 %1, %4, %5\n\tv_fmac_f32 %2, %4, %5\n\tv_fmac_f32 %3, %4, %5\n\t"
#define F4x4 F4 F4 F4 F4

__global__ void probe(float* out, long long* cyc, float x, float w) {
  float a = threadIdx.x * 1e-3f, b = a + 1, c = a + 2, d = a + 3;
  long long t0, t1, t2, t3, t4;
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) asm volatile(F16 : "+v"(a) : "v"(x), "v"(w));
  t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) asm volatile("s_nop 1\n\t" D16 : "+v"(a) : "v"(x), "v"(w));
  t2 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) asm volatile(F2x8 : "+v"(a), "+v"(b) : "v"(x), "v"(w));
  t3 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) asm volatile(F4x4 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  t4 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a + b + c + d;
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
    cyc[3] = t4 - t3;
  }
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 1024 * 4);
  hipMalloc(&cyc, 8 * 8);
  long long h[4];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, 1.0001f, 0.999f);
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  }
  printf("{\"plain_chain_cyc_per_fma\": %.2f, \"dpp_chain_cyc_per_fma\": %.2f, \"two_chains_cyc_per_fma\": %.2f, "
         "\"four_chains_cyc_per_fma\": %.2f}\n",
         h[0] / 1024.0, h[1] / 1024.0, h[2] / 1024.0, h[3] / 1024.0);
  return 0;
}
