// mzh_search.hip -- fused batched MuZero search + batched MLP inference kernels (gfx950).
//
// One workgroup (256 threads = 4 waves) owns R = 16*MT roots and runs ALL of their simulations:
//   select  : 8 lanes per root, one lane per child; fp64 Q / UCB exactly as MCTS/node.py:72-123,
//             6-way argmax + tie detection by shuffles/ballot inside the 8-lane group
//   expand  : recurrent_inference for the R pending leaves as fp32 MFMA GEMMs (mzh_device.h)
//   backup  : one lane per root walks the LDS path leaf -> root (MCTS/node.py:53-70)
// Roots are independent (one owner per tree): no atomics, no inter-workgroup traffic, one launch
// per search.  Trees live in HBM as flat SoA blocks (one 160-B block per expanded node holding its
// 6 children's N/X/R/P/W); the per-sim path, per-root min-max, root stats, UCB table and the MLP
// activations live in LDS.  Weights stream from L2 (shared by every workgroup of an XCD).
#include "mzh_device.h"
#include "mzh_internal.h"

// ------------------------------------------------------------------------------------------
// tree block: the 6 children of one expanded node (+2 pad lanes)
// ------------------------------------------------------------------------------------------
struct __align__(16) MzhBlock {
  uint16_t N[8];  // child visit counts (node.py:21)
  int16_t X[8];   // expanded-node index of the child, -1 = leaf (node.py:19 is_expanded)
  float R[8];     // child reward (python float of an fp32 value, node.py:25)
  float P[8];     // child prior, fp32 (node.py:16)
  double W[8];    // child summed value, fp64 (node.py:22)
};
static_assert(sizeof(MzhBlock) == 160, "block layout");

template <int R>
struct SearchSmem {
  double rootW[R];
  double mm[R][2];  // MinMaxStats (maximum, minimum)
  double p64[R][8]; // root child priors as fp64 (Dirichlet-mixed or widened fp32)
  int rootN[R];
  int firstTie[R];
  int extra[R];
  int depth[R];
  int leafE[R];
  int leafA[R];
  int steps[R];
  int pad_[R];
};

__device__ __forceinline__ double mzh_normalize(double v, double mx, double mn) {
  if (mx > mn) return (v - mn) / (mx - mn);  // utils_mcts.py:12-16
  return v;
}

// x ** e with numpy semantics for the exponents generate_play_policy can produce
__device__ __forceinline__ double mzh_pow(double x, double e) {
  if (e == __builtin_rint(e) && e >= 1.0 && e <= 5.0) {
    double r = x;
    for (int i = 1; i < (int)e; ++i) r = r * x;
    return r;
  }
  return pow(x, e);
}

template <int R, bool REPLAY>
__global__ __launch_bounds__(MZH_THREADS, 1) void mzh_search_kernel(MzhNet net, MzhSearchParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  MlpSmem<R>& sm = *reinterpret_cast<MlpSmem<R>*>(smem_raw);
  SearchSmem<R>& st = *reinterpret_cast<SearchSmem<R>*>(smem_raw + sizeof(MlpSmem<R>));
  double* table = reinterpret_cast<double*>(smem_raw + sizeof(MlpSmem<R>) + sizeof(SearchSmem<R>));
  uint16_t* path = reinterpret_cast<uint16_t*>(table + ((p.S + 2 + 1) & ~1));

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int root0 = blockIdx.x * R;
  const int nvalid = min(R, p.B - root0);
  const int S = p.S;
  const int PL = S + 1;  // path row length
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;

  for (int i = tid; i < S + 2; i += MZH_THREADS) table[i] = p.table[i];
  if (tid < R) {
    const int r = tid;
    st.rootN[r] = 0;
    st.rootW[r] = 0.0;
    st.firstTie[r] = 0;
    st.extra[r] = 0;
    st.steps[r] = 0;
    if (p.minmax_in && r < nvalid) {
      st.mm[r][0] = p.minmax_in[2 * (root0 + r)];
      st.mm[r][1] = p.minmax_in[2 * (root0 + r) + 1];
    } else {
      st.mm[r][0] = -__builtin_inf();
      st.mm[r][1] = __builtin_inf();
    }
  }

  // ---------------- root: initial_inference (mcts.py:49-50) ----------------
  if (!REPLAY) {
    for (int i = tid; i < R * p.kin; i += MZH_THREADS) {
      const int r = i / p.kin, k = i - r * p.kin;
      sm.x[r * MZH_LD64 + k] = (r < nvalid && k < p.in_dim) ? p.obs[(size_t)(root0 + r) * p.in_dim + k] : 0.0f;
    }
    __syncthreads();
    mzh_mlp_initial<R>(sm, net, wave, lane);
    for (int i = tid; i < R * MZH_H; i += MZH_THREADS) {
      const int r = i >> 6, k = i & 63;
      if (r < nvalid) p.htree[((size_t)(root0 + r) * p.E) * MZH_H + k] = sm.x[r * MZH_LD64 + k];
    }
  } else {
    if (tid < R * 8) {
      const int r = tid >> 3, c = tid & 7;
      sm.pi[r * 8 + c] = (r < nvalid && c < MZH_A) ? p.rp_root_pi[(size_t)(root0 + r) * MZH_A + c] : 0.0f;
    }
    __syncthreads();
  }
  // root.expand(prior, h, 0) with optional Dirichlet mixing (mcts.py:57-69, 132-152)
  if (tid < R * 8) {
    const int r = tid >> 3, c = tid & 7;
    if (r < nvalid) {
      MzhBlock* b = reinterpret_cast<MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
      const float pr = c < MZH_A ? sm.pi[r * 8 + c] : 0.0f;
      b->N[c] = 0;
      b->X[c] = -1;
      b->R[c] = 0.0f;
      b->P[c] = pr;
      b->W[c] = 0.0;
      if (c < MZH_A) {
        double v = (double)pr;
        if (noised) {
          const float scaled = (float)(1.0 - p.eps) * pr;  // (1-eps) * prob, float32 array
          v = (double)scaled + p.eps * p.noise[(size_t)(root0 + r) * MZH_A + c];
        }
        st.p64[r][c] = v;
      }
    }
  }
  __syncthreads();

  for (int s = 0; s < S; ++s) {
    // ---------------- Phase 1: select (mcts.py:75-86; node.py:72-123) ----------------
    if (tid < R * 8) {
      const int r = tid >> 3, c = tid & 7, gbase = lane & ~7;
      if (r < nvalid) {
        const MzhBlock* tb = reinterpret_cast<const MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
        const double mmax = st.mm[r][0], mmin = st.mm[r][1];
        int firstTie = st.firstTie[r];
        int extra = st.extra[r];
        const int tie = p.tie_idx ? p.tie_idx[root0 + r] : 0;
        int e = 0, Np = st.rootN[r], depth = 0, pick = 0;
        while (true) {
          const MzhBlock* b = tb + e;
          int Nc = 0, Xc = -1;
          float ucb = -__builtin_inff();
          if (c < MZH_A) {
            Nc = b->N[c];
            Xc = b->X[c];
            const float Rc = b->R[c];
            const float Pc = b->P[c];
            const double Wc = b->W[c];
            float q32 = 0.0f;
            if (Nc > 0) q32 = (float)mzh_normalize((double)Rc + disc * (Wc / (double)Nc), mmax, mmin);
            const double w = table[Np] / (double)(Nc + 1);
            float u32;
            if (e == 0 && noised)
              u32 = (float)(st.p64[r][c] * w);
            else if (p.np1)
              u32 = (float)((double)Pc * w);
            else
              u32 = Pc * (float)w;
            ucb = q32 + u32;
          }
          float m = ucb;
#pragma unroll
          for (int o = 1; o < 8; o <<= 1) {
            const float t = __shfl_xor(m, o);
            m = t > m ? t : m;
          }
          const unsigned long long bal = __ballot(c < MZH_A && ucb == m);
          const unsigned mask = (unsigned)(bal >> gbase) & 0x3Fu;
          const int cnt = __popc(mask);
          if (cnt == 1) {
            pick = __ffs(mask) - 1;
          } else if (!firstTie && cnt == MZH_A) {
            pick = tie;  // np.random.choice over the 6-way argmax set (host pre-drawn)
            firstTie = 1;
          } else {
            pick = __ffs(mask) - 1;
            extra += 1;
          }
          const int Nn = __shfl(Nc, gbase + pick);
          const int Xn = __shfl(Xc, gbase + pick);
          if (c == 0) path[r * PL + depth] = (uint16_t)(e * 8 + pick);
          depth++;
          if (Xn < 0) break;
          e = Xn;
          Np = Nn;
        }
        if (c == 0) {
          st.depth[r] = depth;
          st.leafE[r] = e;
          st.leafA[r] = pick;
          st.steps[r] += depth;
          st.firstTie[r] = firstTie;
          st.extra[r] = extra;
        }
      }
    }
    __syncthreads();

    // ---------------- Phase 2: expand via the network (mcts.py:88-106) ----------------
    if (!REPLAY) {
      for (int i = tid; i < R * 16; i += MZH_THREADS) {
        const int r = i >> 4, qd = i & 15;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < nvalid)
          v = reinterpret_cast<const float4*>(p.htree)[((size_t)(root0 + r) * p.E + st.leafE[r]) * 16 + qd];
        float* d = &sm.x[r * MZH_LD64 + qd * 4];
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
      if (tid < R) sm.act[tid] = tid < nvalid ? st.leafA[tid] : 0;
      __syncthreads();
      mzh_mlp_recurrent<R>(sm, net, wave, lane);
      for (int i = tid; i < R * 16; i += MZH_THREADS) {
        const int r = i >> 4, qd = i & 15;
        if (r < nvalid) {
          const float* src = &sm.x[r * MZH_LD64 + qd * 4];
          reinterpret_cast<float4*>(p.htree)[((size_t)(root0 + r) * p.E + s + 1) * 16 + qd] =
              make_float4(src[0], src[1], src[2], src[3]);
        }
      }
    } else {
      if (tid < R * 8) {
        const int r = tid >> 3, c = tid & 7;
        sm.pi[r * 8 + c] = (r < nvalid && c < MZH_A) ? p.rp_pi[((size_t)(root0 + r) * S + s) * MZH_A + c] : 0.0f;
      }
      if (tid < R) {
        sm.value[tid] = tid < nvalid ? p.rp_value[(size_t)(root0 + tid) * S + s] : 0.0f;
        sm.reward[tid] = tid < nvalid ? p.rp_reward[(size_t)(root0 + tid) * S + s] : 0.0f;
      }
      __syncthreads();
    }

    // ---------------- Phase 3: expand bookkeeping + backup (node.py:30-70) ----------------
    if (tid < R * 8) {
      const int r = tid >> 3, c = tid & 7;
      if (r < nvalid) {
        MzhBlock* tb = reinterpret_cast<MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
        const int enew = s + 1;
        MzhBlock* nb = tb + enew;
        nb->N[c] = 0;
        nb->X[c] = -1;
        nb->R[c] = 0.0f;
        nb->P[c] = c < MZH_A ? sm.pi[r * 8 + c] : 0.0f;
        nb->W[c] = 0.0;
        if (c == 0) {
          const int le = st.leafE[r], la = st.leafA[r];
          const float rew = sm.reward[r];
          tb[le].X[la] = (int16_t)enew;
          tb[le].R[la] = rew;
          double value = (double)sm.value[r];
          double mmax = st.mm[r][0], mmin = st.mm[r][1];
          const int depth = st.depth[r];
          for (int j = depth - 1; j >= 0; --j) {
            const int slot = path[r * PL + j];
            MzhBlock* b = tb + (slot >> 3);
            const int a = slot & 7;
            const double rw = (j == depth - 1) ? (double)rew : (double)b->R[a];
            const double W = b->W[a] + value;
            const int N = b->N[a] + 1;
            b->W[a] = W;
            b->N[a] = (uint16_t)N;
            const double q = rw + disc * (W / (double)N);
            mmax = q > mmax ? q : mmax;
            mmin = q < mmin ? q : mmin;
            value = rw + disc * value;
          }
          const double W = st.rootW[r] + value;
          const int N = st.rootN[r] + 1;
          st.rootW[r] = W;
          st.rootN[r] = N;
          const double q = 0.0 + disc * (W / (double)N);  // root rwd = 0.0
          mmax = q > mmax ? q : mmax;
          mmin = q < mmin ? q : mmin;
          st.mm[r][0] = mmax;
          st.mm[r][1] = mmin;
        }
      }
    }
    __syncthreads();
  }

  // ---------------- results (mcts.py:111-126, 154-176) ----------------
  if (tid < R * 8) {
    const int r = tid >> 3, c = tid & 7;
    if (r < nvalid && c == 0) {
      const int root = root0 + r;
      const MzhBlock* b0 = reinterpret_cast<const MzhBlock*>(p.tree) + (size_t)root * p.E;
      int vis[MZH_A];
      for (int a = 0; a < MZH_A; ++a) {
        vis[a] = b0->N[a];
        p.visits[(size_t)root * MZH_A + a] = vis[a];
      }
      if (p.root_q) p.root_q[root] = st.rootN[r] == 0 ? 0.0 : st.rootW[r] / (double)st.rootN[r];
      if (p.minmax_out) {
        p.minmax_out[2 * root] = st.mm[r][0];
        p.minmax_out[2 * root + 1] = st.mm[r][1];
      }
      if (p.extra_ties) p.extra_ties[root] = st.extra[r];
      if (p.sel_steps) p.sel_steps[root] = st.steps[r];
      if (p.latent && S > 0) {
        const int d = st.depth[r];
        for (int j = 0; j < d; ++j) p.latent[(size_t)root * PL + j] = path[r * PL + j] & 7;
        for (int j = d; j < PL; ++j) p.latent[(size_t)root * PL + j] = -1;
      }
      if (p.latent_len) p.latent_len[root] = S > 0 ? st.depth[r] : 0;
      if (p.pi || p.action) {
        double v[MZH_A];
        for (int a = 0; a < MZH_A; ++a) v[a] = (double)vis[a];
        if (p.temperature > 0.0) {
          double ex = 1.0 / p.temperature;
          ex = ex < 5.0 ? ex : 5.0;  // max(1.0, min(5.0, 1/T))
          ex = ex > 1.0 ? ex : 1.0;
          for (int a = 0; a < MZH_A; ++a) v[a] = mzh_pow(v[a], ex);
        }
        double sum = 0.0;
        for (int a = 0; a < MZH_A; ++a) sum = sum + v[a];
        double pi[MZH_A];
        for (int a = 0; a < MZH_A; ++a) pi[a] = v[a] / sum;
        if (p.pi)
          for (int a = 0; a < MZH_A; ++a) p.pi[(size_t)root * MZH_A + a] = pi[a];
        int act = 0;
        if (p.deterministic || !p.action_u) {
          for (int a = 1; a < MZH_A; ++a)
            if (vis[a] > vis[act]) act = a;
        } else {
          double cdf[MZH_A];
          double acc = 0.0;
          for (int a = 0; a < MZH_A; ++a) {
            acc = acc + pi[a];
            cdf[a] = acc;
          }
          const double last = cdf[MZH_A - 1];
          const double u = p.action_u[root];
          act = MZH_A - 1;
          for (int a = 0; a < MZH_A; ++a) {
            if (cdf[a] / last > u) {
              act = a;
              break;
            }
          }
        }
        if (p.action) p.action[root] = act;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// standalone batched inference kernels (MuZeroNet.initial_inference / recurrent_inference)
// ------------------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(MZH_THREADS, 1) void mzh_initial_kernel(MzhNet net, MzhInferParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  MlpSmem<R>& sm = *reinterpret_cast<MlpSmem<R>*>(smem_raw);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * R;
  const int nvalid = min(R, p.B - row0);
  for (int i = tid; i < R * p.kin; i += MZH_THREADS) {
    const int r = i / p.kin, k = i - r * p.kin;
    sm.x[r * MZH_LD64 + k] = (r < nvalid && k < p.in_dim) ? p.x[(size_t)(row0 + r) * p.in_dim + k] : 0.0f;
  }
  __syncthreads();
  mzh_mlp_initial<R>(sm, net, wave, lane);
  mzh_store_outputs<R>(sm, p, row0, nvalid, net.support, false);
}

template <int R>
__global__ __launch_bounds__(MZH_THREADS, 1) void mzh_recurrent_kernel(MzhNet net, MzhInferParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  MlpSmem<R>& sm = *reinterpret_cast<MlpSmem<R>*>(smem_raw);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * R;
  const int nvalid = min(R, p.B - row0);
  for (int i = tid; i < R * MZH_H; i += MZH_THREADS) {
    const int r = i >> 6, k = i & 63;
    sm.x[r * MZH_LD64 + k] = r < nvalid ? p.x[(size_t)(row0 + r) * MZH_H + k] : 0.0f;
  }
  if (tid < R) sm.act[tid] = tid < nvalid ? p.action[row0 + tid] : 0;
  __syncthreads();
  mzh_mlp_recurrent<R>(sm, net, wave, lane);
  mzh_store_outputs<R>(sm, p, row0, nvalid, net.support, true);
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <int R>
static size_t search_smem_bytes(int S) {
  size_t b = sizeof(MlpSmem<R>) + sizeof(SearchSmem<R>);
  b += sizeof(double) * (size_t)((S + 2 + 1) & ~1);
  b += sizeof(uint16_t) * (size_t)R * (size_t)(S + 1);
  return (b + 15) & ~(size_t)15;
}

size_t mzh_search_smem_bytes(int R, int S) { return R == 32 ? search_smem_bytes<32>(S) : search_smem_bytes<16>(S); }

template <int R, bool REPLAY>
static hipError_t launch_search_t(const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const size_t smem = search_smem_bytes<R>(p.S);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mzh_search_kernel<R, REPLAY>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int grid = (p.B + R - 1) / R;
  hipLaunchKernelGGL((mzh_search_kernel<R, REPLAY>), dim3(grid), dim3(MZH_THREADS), smem, stream, net, p);
  return hipGetLastError();
}

hipError_t mzh_launch_search(int R, bool replay, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  if (R == 32) return replay ? launch_search_t<32, true>(net, p, stream) : launch_search_t<32, false>(net, p, stream);
  return replay ? launch_search_t<16, true>(net, p, stream) : launch_search_t<16, false>(net, p, stream);
}

template <int R>
static hipError_t launch_infer_t(bool recurrent, const MzhNet& net, const MzhInferParams& p, hipStream_t stream) {
  const size_t smem = (sizeof(MlpSmem<R>) + 15) & ~(size_t)15;
  const void* fn = recurrent ? reinterpret_cast<const void*>(&mzh_recurrent_kernel<R>)
                             : reinterpret_cast<const void*>(&mzh_initial_kernel<R>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int grid = (p.B + R - 1) / R;
  if (recurrent)
    hipLaunchKernelGGL((mzh_recurrent_kernel<R>), dim3(grid), dim3(MZH_THREADS), smem, stream, net, p);
  else
    hipLaunchKernelGGL((mzh_initial_kernel<R>), dim3(grid), dim3(MZH_THREADS), smem, stream, net, p);
  return hipGetLastError();
}

hipError_t mzh_launch_infer(int R, bool recurrent, const MzhNet& net, const MzhInferParams& p, hipStream_t stream) {
  return R == 32 ? launch_infer_t<32>(recurrent, net, p, stream) : launch_infer_t<16>(recurrent, net, p, stream);
}
