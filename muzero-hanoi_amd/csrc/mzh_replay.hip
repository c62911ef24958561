// mzh_replay.hip -- prioritised replay with the priorities resident in HBM:
// Buffer.priority_sample's draw and batch gather (buffer.py:89-112) and Buffer.update_priorities
// (buffer.py:127-134) for the reference's defaults (priority exponent 1, importance exponent 0).
//
// The draw has to pick what np.random.choice(np.arange(n), m, replace=True, p=P) picks from the same
// uniforms: RandomState.choice forms cdf = float64(P).cumsum(), cdf /= cdf[-1], searchsorted(u, 'right'),
// with P = p / np.sum(p) in float32.  Two order-sensitive sums decide the result:
//  * np.sum over float32 (NumPy 2.x add.reduce): 0 + the pairwise sums of consecutive 8,192-element
//    buffers, a buffer's pairwise sum splitting n at n/2 rounded down to a multiple of 8 until a block
//    has <= 128 elements, each block summed with 8 interleaved accumulators (NumPy's pairwise_sum,
//    loops_utils.h.src; restated in oracle/replay_ref.py and pinned against np.sum by tests/test_replay.py).
//    Here 8 lanes sum a block (one accumulator each); a full buffer is a perfect tree of 64 blocks, combined
//    by one wave's xor butterfly; the last, partial buffer's tree is walked by one lane (its path in
//    register bits).
//  * the cumsum is a sequential float64 chain.  When every non-zero P_i is >= 2^-28 its float32 ulp is
//    >= 2^-51, so every P_i is an integer multiple of 2^-51; with the total below 4 every partial sum (of
//    any subset) is such a multiple below 4, an exact float64 value, so every float64 addition is exact
//    and any order gives NumPy's values: the workgroup scans segment sums in float64.  Otherwise (a
//    probability below 2^-28 next to larger ones) one lane runs NumPy's chain through LDS tiles.
// The search runs on a 4,096-entry LDS sample of the normalised cdf, then on a window of <= 16 entries
// loaded at once (binary steps in HBM first above 65,536 transitions); the sampled rows are gathered by
// the whole workgroup, every load independent.  One 1,024-thread workgroup: at the
// reference's buffer (50,000 transitions) the draw is a few latency-bound passes over 200 KB; one launch
// replaces the host's NumPy passes and the index and weight uploads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mzh_device.h"
#include "mzh_train.h"

namespace {

constexpr int RT = 1024;                  // threads of the one workgroup
constexpr int NWAVE = RT / 64;
constexpr int CHUNK = 8192;               // NumPy's reduction buffer (elements)
constexpr int BLOCK = 128;                // NumPy's PW_BLOCKSIZE
constexpr int LEAVES = CHUNK / BLOCK;     // a full buffer is a perfect tree of 64 blocks of 128
constexpr int GROUP = 32;                 // full buffers per pass
constexpr int PMAX = 128;                 // blocks of a partial buffer (each >= 64 elements)
constexpr int FT = 2048;                  // sequential-chain tile
constexpr int NC = 4096;                  // LDS sample of the cdf
constexpr int LIN = 16;                   // final search window, loaded at once
constexpr float kMinExact = 3.7252902984e-09f;  // 2^-28: float32 ulp >= 2^-51
constexpr double kMaxTotal = 4.0;               // multiples of 2^-51 below 4 are exact float64 values

__device__ __forceinline__ int pw_split(int n) {
  const int h = n / 2;
  return h - h % 8;
}

union ReplayPhase {
  float full[GROUP * LEAVES];  // block sums of full buffers
  struct {
    float q[FT];
    double c[FT];
  } f;            // sequential cumsum tiles
  double cn[NC];  // cdf sample
};

struct ReplayLds {
  ReplayPhase u;
  double wtot[4][NWAVE];
  double wpre[4 * NWAVE + 1];
  int sidx[MZR_MAX_BATCH];
  int poff[PMAX];
  short plen[PMAX];
  char ppop[PMAX];
  float pval[PMAX];
  float cval[GROUP];
  float saved[16];
  int npart;
  float total;
};

// NumPy's block sum (n <= 128) on 8 consecutive lanes: lane j holds accumulator r[j] (elements j, j + 8, ...
// below n - n % 8); an xor butterfly over the 8 forms ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) (every lane of the
// group ends with it: each sum's two operands are the same on both lanes), then the tail.  Returns the
// sum on all 8 lanes.
__device__ __forceinline__ float block_sum8(const float* blk, int len, int j) {
  const int n8 = len - len % 8;
  float r = 0.f;
  if (len >= 8) {
    float v[15];
#pragma unroll
    for (int q = 0; q < 15; ++q) v[q] = 8 + j + 8 * q < n8 ? blk[8 + j + 8 * q] : 0.f;
    r = blk[j];
#pragma unroll
    for (int q = 0; q < 15; ++q)
      if (8 + j + 8 * q < n8) r += v[q];
  }
  r = r + __shfl_xor(r, 1);
  r = r + __shfl_xor(r, 2);
  r = r + __shfl_xor(r, 4);
  float res = 0.f;
  int i = 0;
  if (len >= 8) {
    res = r;
    i = n8;
  }
  for (; i < len; ++i) res += blk[i];
  return res;
}

// the node at the end of `path` (bit k: right child at depth k) of the pairwise tree over [0, L)
__device__ __forceinline__ void pw_node(int L, unsigned path, int d, int& o, int& len) {
  o = 0;
  len = L;
  for (int k = 0; k < d; ++k) {
    const int h = pw_split(len);
    if ((path >> k) & 1u) {
      o += h;
      len -= h;
    } else {
      len = h;
    }
  }
}

// the blocks of the pairwise tree over [0, L) in order (one lane): each block's offset and length, and how
// many of the tree's additions complete right after it (the right turns that end at it)
__device__ void pw_blocks(ReplayLds& Ls, int base, int L) {
  unsigned path = 0;  // bit k: right child at depth k
  int d = 0, o = 0, len = L, cur = 0;
  while (len > BLOCK) {
    len = pw_split(len);
    ++d;
  }
  for (;;) {
    Ls.poff[cur] = base + o;
    Ls.plen[cur] = (short)len;
    int k = d - 1;
    while (k >= 0 && ((path >> k) & 1u)) --k;
    Ls.ppop[cur] = (char)(d - 1 - k);
    ++cur;
    if (k < 0) break;
    path = (path & ((1u << k) - 1u)) | (1u << k);  // the deepest left turn becomes a right turn
    d = k + 1;
    pw_node(L, path, d, o, len);
    while (len > BLOCK) {
      len = pw_split(len);
      ++d;
    }
  }
  Ls.npart = cur;
}

// the tree's value from the block sums: a stack machine (push each block, then its completed additions,
// left + right)
__device__ float pw_combine(ReplayLds& Ls) {
  int sp = 0;
  for (int l = 0; l < Ls.npart; ++l) {
    float v = Ls.pval[l];
    for (int c = Ls.ppop[l]; c > 0; --c) v = Ls.saved[--sp] + v;
    Ls.saved[sp++] = v;
  }
  return Ls.saved[0];
}

// words sub, sub + tpr, ... of row r of src (w words per row) to row o of dst, 4 loads in flight
__device__ __forceinline__ void copy_row(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int w,
                                         size_t r, size_t o, int sub, int tpr) {
  for (int c0 = sub; c0 < w; c0 += 4 * tpr) {
    uint32_t v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = c0 + t * tpr;
      v[t] = c < w ? src[r * w + c] : 0u;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = c0 + t * tpr;
      if (c < w) dst[o * w + c] = v[t];
    }
  }
}

#ifdef MZH_STAMPS
// diagnostic build: lane 0 records s_memtime after each phase into status[2..9] (the caller sizes status)
#define MZR_STAMP(i) \
  if (tid == 0) stamp[i] = __builtin_amdgcn_s_memtime();
#else
#define MZR_STAMP(i)
#endif

// one float64 through DPP (both halves).  ROWS == 0xF: lanes without a source read +0.0 (bound_ctrl);
// else the rows outside ROWS keep the +0.0 `old`
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  int lo, hi;
  if (ROWS == 0xF) {
    lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, ROWS, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, ROWS, 0xF, true);
  } else {
    lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xF, false);
    hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
  }
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// inclusive scan over the wave in lane order: row_shr 1, 2, 4, 8 within rows of 16, then row_bcast 15 / 31
// (only sums that are exact in any order are scanned here)
__device__ __forceinline__ double wave_scan(double v) {
  v += dpp_f64<0x111, 0xF>(v);
  v += dpp_f64<0x112, 0xF>(v);
  v += dpp_f64<0x114, 0xF>(v);
  v += dpp_f64<0x118, 0xF>(v);
  v += dpp_f64<0x142, 0xA>(v);
  v += dpp_f64<0x143, 0xC>(v);
  return v;
}

// a / b (a >= 0, b > 0, the quotient in [0, 1] and not subnormal) from y = RN(1/b): Markstein's correction,
// equal to IEEE division there (mzh_tree.h mzh_div; tests/test_markstein.py)
__device__ __forceinline__ double rdiv(double a, double b, double y) {
  const double q = a * y;
  return __builtin_fma(__builtin_fma(-q, b, a), y, q);
}

__global__ __launch_bounds__(RT) void replay_sample_kernel(mzh_replay_args a) {
  __shared__ ReplayLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n = a.n, m = a.m;
  const float* p = a.prio;
#ifdef MZH_STAMPS
  unsigned long long stamp[8] = {};
#endif
  MZR_STAMP(0)

  // ---- np.sum(p): 0 + pairwise(buffer 0) + pairwise(buffer 1) + ...  The last, partial buffer's blocks
  // come from a walk of its tree by the last lane, overlapped with the full buffers' block sums.
  const int nfull = n / CHUNK, rem = n - nfull * CHUNK;
  if (tid == RT - 1 && rem > 0) pw_blocks(L, nfull * CHUNK, rem);
  float tot = 0.f;  // lane 0's running sum
  for (int c0 = 0; c0 < nfull; c0 += GROUP) {
    const int nc = min(GROUP, nfull - c0);
    for (int l = tid >> 3; l < nc * LEAVES; l += RT / 8)
      L.u.full[l] = block_sum8(p + (size_t)c0 * CHUNK + (size_t)l * BLOCK, BLOCK, tid & 7);
    __syncthreads();
    for (int c = wave; c < nc; c += NWAVE) {  // a full buffer's perfect tree: pairs, then pairs of pairs, ...
      float v = L.u.full[c * LEAVES + lane];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) v = v + __shfl_xor(v, off);
      if (lane == 0) L.cval[c] = v;
    }
    __syncthreads();
    if (tid == 0)
      for (int c = 0; c < nc; ++c) tot += L.cval[c];
  }
  __syncthreads();
  MZR_STAMP(1)
  if (rem > 0) {
    for (int l = tid >> 3; l < L.npart; l += RT / 8)
      L.pval[l] = block_sum8(p + L.poff[l], L.plen[l], tid & 7);
    __syncthreads();
    if (tid == 0) tot += pw_combine(L);
  }
  if (tid == 0) L.total = tot;
  __syncthreads();
  const float s = L.total;
  MZR_STAMP(2)

  // ---- P_i = p_i / s and the cdf in one pass.  A sub-tile is 4 consecutive elements per lane over the
  // workgroup (float4 loads coalesce); a lane's sum, a wave scan and the waves' totals through LDS give the
  // cdf at every 4th element (cdf4, the only values stored: the search replays a group's 4 additions), NS
  // sub-tiles per barrier.  On the exact path every
  // partial sum of the P_i is a multiple of 2^-51 below 4, so these float64 additions in any order are
  // exact and the prefixes are NumPy's cumsum values; else (or if invalid) the values written here are
  // replaced below.  Quotients by Markstein from y = RN(1/s) (mzh_fdiv: exact unless an operand is tiny,
  // then the wave divides in IEEE).
  constexpr int NS = 4, SUB = RT * 4;
  const float y = 1.0f / s;
  int valid = (s > 0.f && s < __builtin_inff()) ? 1 : 0, exact = 1;
  double carry = 0.0;
  static_assert(NS * NWAVE == 64, "one wave scans the wave totals");
  // a tile's elements (those past n read as 0: P = 0 changes no sum or flag); the next tile's are loaded
  // while this one is processed
  auto load_tile = [&](int t0, float (&x)[NS][4]) {
    const bool whole = t0 + NS * SUB <= n;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int i = t0 + j * SUB + 4 * tid;
      if (whole || i + 4 <= n) {
        const float4 v = *reinterpret_cast<const float4*>(p + i);
        x[j][0] = v.x;
        x[j][1] = v.y;
        x[j][2] = v.z;
        x[j][3] = v.w;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) x[j][t] = i + t < n ? p[i + t] : 0.f;
      }
    }
  };
  float xn[NS][4];
  load_tile(0, xn);
  for (int t0 = 0; t0 < n; t0 += NS * SUB) {
    float x[NS][4];
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) x[j][t] = xn[j][t];
    if (t0 + NS * SUB < n) load_tile(t0 + NS * SUB, xn);
    bool slow = false;
    float q[NS][4];
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) q[j][t] = mzh_fdiv(x[j][t], s, y, slow);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(slow) != 0, 0)) {
      asm volatile("" ::: "memory");  // keeps the IEEE divisions behind the branch (not speculated)
#pragma unroll
      for (int j = 0; j < NS; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) q[j][t] = x[j][t] / s;
    }
    double run[NS], w[NS];
    bool ok = true, ex = true;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      run[j] = 0.0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float v = q[j][t];
        ok &= (v >= 0.f) & (v <= 1.f);  // else NaN, negative, or a sum that overflowed
        ex &= (v == 0.f) | (v >= kMinExact);
        run[j] += (double)v;
      }
      w[j] = run[j];
    }
    valid &= ok ? 1 : 0;
    exact &= ex ? 1 : 0;
#pragma unroll
    for (int j = 0; j < NS; ++j) w[j] = wave_scan(w[j]);
    if (lane == 63) {
#pragma unroll
      for (int j = 0; j < NS; ++j) L.wtot[j][wave] = w[j];
    }
    __syncthreads();
    if (wave == 0) {  // the NS x 16 wave totals in (sub-tile, wave) order: one more wave scan
      const double t = L.wtot[lane >> 4][lane & 15];
      const double v = wave_scan(t);
      L.wpre[lane] = v - t;  // exclusive
      if (lane == 63) L.wpre[64] = v;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      // the cdf at this lane's 4th element (elements past n added 0): cdf4[g] = cdf[min(4g + 3, n - 1)]
      const int i = t0 + j * SUB + 4 * tid;
      if (i < n) a.cdf[i >> 2] = carry + L.wpre[j * NWAVE + wave] + w[j];
    }
    carry += L.wpre[64];
  }
  valid = __syncthreads_and(valid);
  exact = __syncthreads_and(exact) && carry < kMaxTotal;
  MZR_STAMP(3)

  if (valid && !exact) {  // NumPy's chain, out[0] = P_0, out[i] = out[i-1] + P_i, through LDS tiles
    double c = 0.0;
    for (int t0 = 0; t0 < n; t0 += FT) {
      const int tn = min(FT, n - t0);
      for (int i = tid; i < tn; i += RT) L.u.f.q[i] = p[t0 + i] / s;
      __syncthreads();
      if (tid == 0) {
        for (int i = 0; i < tn; ++i) {
          c += (double)L.u.f.q[i];
          L.u.f.c[i >> 2] = c;  // a group's last write is its 4th element (or element n - 1)
        }
      }
      __syncthreads();
      for (int g = tid; g < (tn + 3) / 4; g += RT) a.cdf[(t0 >> 2) + g] = L.u.f.c[g];
      __syncthreads();
    }
  }
  if (tid == 0) {
    a.status[0] = valid ? 0 : 1;
    a.status[1] = valid && exact ? 1 : 0;
  }
  __syncthreads();

  MZR_STAMP(4)
  // ---- searchsorted(u, 'right') on cdf / cdf[n-1]: the group of 4 from the LDS sample of cdf4 and a window
  // of cdf4 in HBM, then the element inside the group by replaying its 4 additions from the previous
  // group's value (NumPy's own chain on either path: exact sums, or the sequential values themselves)
  if (valid) {
    const int n4 = (n + 3) >> 2;
    const double last = a.cdf[n4 - 1], ylast = 1.0 / last;  // cdf / last by Markstein (rdiv)
    const int stride = (n4 + NC - 1) / NC, nc = (n4 + stride - 1) / stride;
    for (int jj = tid; jj < nc; jj += RT) L.u.cn[jj] = rdiv(a.cdf[min(n4, (jj + 1) * stride) - 1], last, ylast);
    __syncthreads();
    MZR_STAMP(5)
    for (int k = tid; k < m; k += RT) {
      const double uk = a.u[k];
      int lo = 0, hi = nc - 1;  // the first sample above uk (the last one is 1.0 > uk)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L.u.cn[mid] > uk)
          hi = mid;
        else
          lo = mid + 1;
      }
      int g = lo * stride, e = min(n4, (lo + 1) * stride) - 1;  // the group is in [g, e], cdf4[e] above uk
      while (e - g >= LIN) {
        const int mid = (g + e) >> 1;
        if (rdiv(a.cdf[mid], last, ylast) > uk)
          e = mid;
        else
          g = mid + 1;
      }
      double w[LIN];  // the window at once: the group is g + the number of entries at or below uk
#pragma unroll
      for (int t = 0; t < LIN; ++t) w[t] = g + t < e ? a.cdf[g + t] : 0.0;
      int below = 0;
#pragma unroll
      for (int t = 0; t < LIN; ++t) below += (g + t < e && !(rdiv(w[t], last, ylast) > uk)) ? 1 : 0;
      g += below;
      double c = g > 0 ? a.cdf[g - 1] : 0.0;
      const int i0 = 4 * g, cnt = min(4, n - i0);
      float x[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) x[t] = t < cnt ? p[i0 + t] : 0.f;
      int idx = i0 + cnt - 1;  // the group's last element is above uk
      bool found = false;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < cnt && !found) {
          c += (double)(x[t] / s);
          if (rdiv(c, last, ylast) > uk) {
            idx = i0 + t;
            found = true;
          }
        }
      }
      L.sidx[k] = idx;
      a.indx[k] = idx;
    }
  } else {
    for (int k = tid; k < m; k += RT) {
      L.sidx[k] = 0;
      a.indx[k] = 0;
    }
  }
  __syncthreads();

  MZR_STAMP(6)
  // ---- the sampled rows: `tpr` lanes per sample copy its five rows word by word (no division per word)
  const int tpr = m > RT / 2 ? 1 : (m > RT / 4 ? 2 : (m > RT / 8 ? 4 : (m > RT / 16 ? 8 : 16)));
  const int sub = tid % tpr;
  for (int k = tid / tpr; k < m; k += RT / tpr) {
    const size_t r = (size_t)L.sidx[k], o = (size_t)k;
    copy_row((const uint32_t*)a.states, (uint32_t*)a.out_states, a.d_state, r, o, sub, tpr);
    copy_row((const uint32_t*)a.rwds, (uint32_t*)a.out_rwds, a.U, r, o, sub, tpr);
    copy_row((const uint32_t*)a.actions, (uint32_t*)a.out_actions, 2 * a.U, r, o, sub, tpr);
    copy_row((const uint32_t*)a.pi, (uint32_t*)a.out_pi, a.U * a.A, r, o, sub, tpr);
    copy_row((const uint32_t*)a.returns, (uint32_t*)a.out_returns, a.U, r, o, sub, tpr);
  }
#ifdef MZH_STAMPS
  __syncthreads();
  MZR_STAMP(7)
  if (tid == 0)
    for (int k = 0; k < 8; ++k) a.status[2 + k] = (int32_t)(stamp[k] - stamp[0]);
#endif
}

__global__ __launch_bounds__(RT) void replay_set_priorities_kernel(float* prio, long long size, const int64_t* idx,
                                                                   const float* val, int m, int32_t* status) {
  __shared__ long long sidx[MZR_MAX_BATCH];
  const int tid = threadIdx.x;
  int fin = 1, pos = 0, inr = 1;
  for (int k = tid; k < m; k += RT) {
    const float v = val[k];
    const long long i = idx[k];
    sidx[k] = i;
    if (!isfinite(v)) fin = 0;
    if (v > 0.f) pos = 1;
    if (i < 0 || i >= size) inr = 0;
  }
  fin = __syncthreads_and(fin);
  pos = __syncthreads_or(pos);
  inr = __syncthreads_and(inr);
  const int bad = !(fin && pos) ? 1 : (!inr ? 2 : 0);
  if (tid == 0) status[0] = bad;
  if (bad) return;
  for (int k = tid; k < m; k += RT) {
    const long long i = sidx[k];
    bool later = false;  // NumPy's prio[idx] = val: the last of repeated indices stays
    int j = k + 1;
    for (; j + 8 <= m; j += 8) {
      long long w[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) w[t] = sidx[j + t];
#pragma unroll
      for (int t = 0; t < 8; ++t) later |= w[t] == i;
    }
    for (; j < m; ++j) later |= sidx[j] == i;
    if (!later) prio[i] = val[k];
  }
}

}  // namespace

hipError_t mzr_launch_sample(const mzh_replay_args& a, hipStream_t stream) {
  hipLaunchKernelGGL(replay_sample_kernel, dim3(1), dim3(RT), 0, stream, a);
  return hipGetLastError();
}

hipError_t mzr_launch_set_priorities(float* prio, long long size, const int64_t* idx, const float* val, int m,
                                     int32_t* status, hipStream_t stream) {
  hipLaunchKernelGGL(replay_set_priorities_kernel, dim3(1), dim3(RT), 0, stream, prio, size, idx, val, m, status);
  return hipGetLastError();
}
