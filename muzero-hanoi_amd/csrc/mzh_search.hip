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
// tree block: the 6 children of one expanded node in exactly one 128-byte cache line, so a
// selection level touches one line (L2-resident hot path)
// ------------------------------------------------------------------------------------------
struct MzhNX {
  uint16_t N;  // child visit count (node.py:21)
  int16_t X;   // expanded-node index of the child, -1 = not expanded (node.py:19 is_expanded)
};
struct __align__(128) MzhBlock {
  MzhNX nx[6];  // N and X adjacent: one dword load per child in selection
  float R[6];   // child reward (python float of an fp32 value, node.py:25)
  float P[6];   // child prior, fp32 (node.py:16)
  double W[6];  // child summed value, fp64 (node.py:22)
  uint32_t pad[2];
};
static_assert(sizeof(MzhBlock) == 128, "block layout");
static_assert(__builtin_offsetof(MzhBlock, W) == 72, "block layout");


// the root's 6 children live in LDS for the whole search (every simulation starts there)
struct MzhRootBlk {
  double W[8];
  double P64[8];  // prior as fp64: Dirichlet-mixed (np.float64) or the widened fp32 prior
  float R[8];
  int N[8];
  int X[8];
};

// snapshot of the chosen child's statistics at each depth of the current simulation's path,
// taken during selection so the backup needs no dependent global loads (depth < DC)
struct MzhPathEnt {
  double W;
  float R;
  int N;
};

template <int R>
struct SearchSmem {
  static constexpr int DC = R == 32 ? 16 : 32;
  MzhRootBlk root[R];
  MzhPathEnt pc[R][DC];
  double bval[R][DC];  // value added at each cached path depth (backup value chain)
  double rootW[R];
  double mm[R][4];  // MinMaxStats (maximum, minimum) + normaliser (max - min, RN(1/(max - min)))
  int rootN[R];
  int firstTie[R];
  int extra[R];
  int depth[R];
  int leafE[R];
  int leafA[R];
  int steps[R];
  int pad_[R];
};

// a / b correctly rounded from y = RN(1/b) (Markstein: q = RN(a*y) is within one ulp, the fma
// residual is exact, and one correction step rounds to RN(a/b)); 3 fp64 ops instead of the
// ~12-op div_scale/rcp/fmas/fixup sequence on the select chain.  Equal to `a / b` for every
// finite non-subnormal quotient; checked against true division in tests/test_markstein.py.
__device__ __forceinline__ double mzh_div(double a, double b, double y) {
  const double q = a * y;
  const double r = __builtin_fma(-q, b, a);
  return __builtin_fma(r, y, q);
}

// MinMaxStats.normalize (utils_mcts.py:12-16) with den = max - min, dinv = RN(1/den)
__device__ __forceinline__ double mzh_normalize(double v, bool has, double mn, double den, double dinv) {
  return has ? mzh_div(v - mn, den, dinv) : v;
}

// ucb = fl32(Q) + fl32(U) for one child (node.py:90-123); `tnp` = table[N_parent], inv[k] = RN(1/k)
__device__ __forceinline__ float mzh_ucb(int Nc, double Wc, float Rc, double P64, bool p64_semantics, double tnp,
                                         double disc, bool has, double mn, double den, double dinv,
                                         const double* inv) {
  float q32 = 0.0f;
  if (Nc > 0) q32 = (float)mzh_normalize((double)Rc + disc * mzh_div(Wc, (double)Nc, inv[Nc]), has, mn, den, dinv);
  const double w = mzh_div(tnp, (double)(Nc + 1), inv[Nc + 1]);
  // np.float64 priors (Dirichlet-mixed root) or NumPy-1 promotion: fl32(fl64(prior * w));
  // NumPy-2 with np.float32 priors: fl32(prior * fl32(w))
  const float u32 = p64_semantics ? (float)(P64 * w) : (float)P64 * (float)w;
  return q32 + u32;
}

// MinMaxStats update with the select-side normaliser precomputed (den, RN(1/den))
__device__ __forceinline__ void mzh_mm_set(double* mm, double mx, double mn) {
  mm[0] = mx;
  mm[1] = mn;
  mm[2] = mx - mn;
  mm[3] = mx > mn ? 1.0 / (mx - mn) : 0.0;
}

// argmax over the 6 children held by the 8-lane group, with the reference's tie handling:
// np.random.choice(argmax set) -- the first 6-way tie takes the host-drawn index, any other tie
// is counted (RNG-stream divergence) and resolved to the lowest index.  Branch-free; every lane
// of the group returns the same pick.
__device__ __forceinline__ int mzh_group_pick(float ucb, int c, int lane, int tie, int& firstTie, int& extra) {
  const float m = mzh_max8(ucb);
  const unsigned long long bal = __ballot(c < MZH_A && ucb == m);
  const unsigned mask = (unsigned)(bal >> (lane & ~7)) & 0x3Fu;
  const int cnt = __popc(mask);
  const int first = __ffs(mask) - 1;
  const bool six = (cnt == MZH_A) & (firstTie == 0);
  extra += ((cnt > 1) & !six) ? 1 : 0;
  firstTie |= six ? 1 : 0;
  return six ? tie : first;
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

// One workgroup per CU (all 512 registers per lane): the next simulation's first weight chunks stay
// in flight across the tree phase.  (Two co-resident 16-root workgroups per CU without that prefetch,
// <= 256 registers and 16 cached path depths, measured 11% slower at 8,192 roots: DESIGN.md §3.)
template <int R, bool REPLAY, bool OHL>
__global__ __launch_bounds__(MZH_THREADS, 1) void mzh_search_kernel(MzhNet net, MzhSearchParams p) {
  constexpr int DC = SearchSmem<R>::DC;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  MlpSmem<R>& sm = *reinterpret_cast<MlpSmem<R>*>(smem_raw);
  SearchSmem<R>& st = *reinterpret_cast<SearchSmem<R>*>(smem_raw + sizeof(MlpSmem<R>));
  double* table = reinterpret_cast<double*>(smem_raw + sizeof(MlpSmem<R>) + sizeof(SearchSmem<R>));
  double* inv = table + (p.S + 3);  // inv[k] = RN(1/k), k <= S + 2
  uint16_t* path = reinterpret_cast<uint16_t*>(table + 2 * (p.S + 3));
  // OHL: the dynamics one-hot columns (6 x 256 floats) live in LDS (when the launcher finds room)
  float* ohl = reinterpret_cast<float*>(path + ((R * (p.S + 1) + 7) & ~7));

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int root0 = blockIdx.x * R;
  const int nvalid = min(R, p.B - root0);
  const int S = p.S;
  const int PL = S + 1;  // path row length
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;

  if (OHL)
    for (int i = tid; i < MZH_A * MZH_F; i += MZH_THREADS) ohl[i] = net.dyn0_onehot[i];
  for (int i = tid; i < S + 3; i += MZH_THREADS) {
    table[i] = i < S + 2 ? p.table[i] : 0.0;
    inv[i] = 1.0 / (double)i;  // IEEE division: correctly rounded
  }
  if (tid < R) {
    const int r = tid;
    st.rootN[r] = 0;
    st.rootW[r] = 0.0;
    st.firstTie[r] = 0;
    st.extra[r] = 0;
    st.steps[r] = 0;
    st.depth[r] = 0;
    if (p.minmax_in && r < nvalid) {
      mzh_mm_set(st.mm[r], p.minmax_in[2 * (root0 + r)], p.minmax_in[2 * (root0 + r) + 1]);
    } else {
      mzh_mm_set(st.mm[r], -__builtin_inf(), __builtin_inf());
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
    MzhRootBlk& rb = st.root[r];
    const float pr = (r < nvalid && c < MZH_A) ? sm.pi[r * 8 + c] : 0.0f;
    rb.N[c] = 0;
    rb.X[c] = -1;
    rb.R[c] = 0.0f;
    rb.W[c] = 0.0;
    double v = (double)pr;
    if (noised && r < nvalid && c < MZH_A) {
      const float scaled = (float)(1.0 - p.eps) * pr;  // (1-eps) * prob, float32 array
      v = (double)scaled + p.eps * p.noise[(size_t)(root0 + r) * MZH_A + c];
    }
    rb.P64[c] = v;
  }
  if (tid < R && tid >= nvalid) sm.act[tid] = 0;  // rows beyond the batch: any valid one-hot index
  floatx4 fa[16], fb[16];
  float ba[4], bb[4];
  if (!REPLAY) mzh_mlp_fetch12<R>(sm, net, wave, lane, fa, ba, fb, bb);
  __syncthreads();

  MZH_STAMP_DECL
  for (int s = 0; s < S; ++s) {
    MZH_STAMP(16);
    // ---------------- Phase 1: select (mcts.py:75-86; node.py:72-123) ----------------
    if (tid < R * 8) {
      const int r = tid >> 3, c = tid & 7;
      if (r < nvalid) {
        const MzhBlock* tb = reinterpret_cast<const MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
        const double mmax = st.mm[r][0], mmin = st.mm[r][1], den = st.mm[r][2], dinv = st.mm[r][3];
        const bool has = mmax > mmin;
        int firstTie = st.firstTie[r];
        int extra = st.extra[r];
        const int tie = p.tie_idx ? p.tie_idx[root0 + r] : 0;
        // level 0: the root block (LDS)
        int Nc = 0, Xc = -1;
        double Wc = 0.0;
        float Rc = 0.0f;
        float ucb = -__builtin_inff();
        if (c < MZH_A) {
          const MzhRootBlk& rb = st.root[r];
          Nc = rb.N[c];
          Xc = rb.X[c];
          Wc = rb.W[c];
          Rc = rb.R[c];
          ucb = mzh_ucb(Nc, Wc, Rc, rb.P64[c], noised || p.np1, table[st.rootN[r]], disc, has, mmin, den, dinv, inv);
        }
        int pick = mzh_group_pick(ucb, c, lane, tie, firstTie, extra);
        // the picking lane records the path entry and its own statistics; one shuffle of the
        // packed (N | X << 16) word moves the selection on
        if (c == pick) {
          path[r * PL] = (uint16_t)pick;
          st.pc[r][0] = MzhPathEnt{Wc, Rc, Nc};
        }
        // every lane prefetches its own child's block (the selection's next level is one of
        // them): the block's cache lines are in flight while this level's UCB/argmax completes
        // (unconditional loads -- a lane without a child re-reads a valid block -- so the
        // compiler can count outstanding loads and wait only for the ones a level needs)
        int pf0 = 0;
        pf0 = *reinterpret_cast<const int*>(tb + (Xc >= 0 ? Xc : 0));
        int nx = __shfl((Nc & 0xFFFF) | (Xc << 16), (lane & ~7) + pick);
        int depth = 1, e = 0;

        // deeper levels: tree blocks in HBM (L2); lanes 6, 7 re-read slot 5 and act as
        // unexpanded, unvisited pads (N = 0, X = -1)
        const int cs = c < MZH_A ? c : MZH_A - 1;
        MZH_STAMP(29);
        MZH_LSTAMP_DECL
        while ((nx >> 16) >= 0) {
          MZH_LSTAMP_COUNT();
          e = nx >> 16;
          const int Np = nx & 0xFFFF;
          const MzhBlock* b = tb + e;
          int nxc = *reinterpret_cast<const int*>(&b->nx[cs]);
          Rc = b->R[cs];
          Wc = b->W[cs];
          const float Pc = b->P[cs];
          if (c >= MZH_A) nxc = (int)0xFFFF0000;
          // retire the previous level's prefetch (older than this level's block loads, so no
          // extra wait) -- keeps it in flight inside the loop
          asm volatile("" ::"v"(pf0));
          const int xc = nxc >> 16;
          pf0 = *reinterpret_cast<const int*>(tb + (xc >= 0 ? xc : e));
          Nc = nxc & 0xFFFF;
          MZH_LSTAMP(0);
          ucb = c < MZH_A ? mzh_ucb(Nc, Wc, Rc, (double)Pc, p.np1, table[Np], disc, has, mmin, den, dinv, inv)
                          : -__builtin_inff();
          MZH_LSTAMP(1);
          pick = mzh_group_pick(ucb, c, lane, tie, firstTie, extra);
          MZH_LSTAMP(2);
          if (c == pick) {
            path[r * PL + depth] = (uint16_t)(e * 8 + pick);
            if (depth < DC) st.pc[r][depth] = MzhPathEnt{Wc, Rc, Nc};
          }
          nx = __shfl(nxc, (lane & ~7) + pick);
          depth++;
          MZH_LSTAMP(3);
        }
        MZH_LSTAMP_FLUSH(24);
        MZH_STAMP(30);
        asm volatile("" ::"v"(pf0));
        if (c == 0) {
          st.depth[r] = depth;
          st.leafE[r] = e;
          st.leafA[r] = pick;
          st.steps[r] += depth;
          st.firstTie[r] = firstTie;
          st.extra[r] = extra;
        }
        if (!REPLAY) {
          // MLP input for this root: the parent's latent (mcts.py:89-92) and the leaf's move
          // MLP input: the leaf's parent latent (mcts.py:89-92).  The node expanded by the previous
          // simulation (index s; the root at s = 0) is still in sm.x as that MLP's output.
          if (e != s) {
            const floatx4* hsrc = reinterpret_cast<const floatx4*>(p.htree) + ((size_t)(root0 + r) * p.E + e) * 16 + c * 2;
            const floatx4 h0 = hsrc[0], h1 = hsrc[1];
            float* d = &sm.x[r * MZH_LD64 + c * 8];
            d[0] = h0[0]; d[1] = h0[1]; d[2] = h0[2]; d[3] = h0[3];
            d[4] = h1[0]; d[5] = h1[1]; d[6] = h1[2]; d[7] = h1[3];
          }
          if (c == 0) sm.act[r] = pick;
        }
      }
    }
    MZH_STAMP(17);
    __syncthreads();
    MZH_STAMP(18);

    // ---------------- Phase 2: expand via the network (mcts.py:88-106) ----------------
    if (!REPLAY) {
      MZH_STAMP(19);
      mzh_mlp_recurrent_body<R, true>(sm, net, wave, lane, fa, ba, fb, bb, OHL ? ohl : net.dyn0_onehot);
      MZH_STAMP(20);
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

    MZH_STAMP(21);
    // ---------------- Phase 3: expand bookkeeping + backup (node.py:30-70) ----------------
    // Lane 0 of each root's group runs the value chain leaf -> root (two fp64 ops per level, the
    // only serial part); the 8 lanes then update the cached path nodes in parallel and reduce
    // the MinMaxStats candidates (max/min are exact and order-free).
    if (tid < R * 8) {
      const int r = tid >> 3, c = tid & 7;
      if (r < nvalid) {
        MzhBlock* tb = reinterpret_cast<MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
        MzhRootBlk& rb = st.root[r];
        const int enew = s + 1;
        if (!REPLAY) {
          // the new node's latent (read back when one of its children is expanded -- usually
          // within a few simulations on the deepening path, so it stays cacheable)
          const float* src = &sm.x[r * MZH_LD64 + c * 8];
          floatx4* dst = reinterpret_cast<floatx4*>(p.htree) + ((size_t)(root0 + r) * p.E + enew) * 16 + c * 2;
          const floatx4 v0 = {src[0], src[1], src[2], src[3]}, v1 = {src[4], src[5], src[6], src[7]};
          dst[0] = v0;
          dst[1] = v1;
        }
        MzhBlock* nb = tb + enew;  // the new expanded node's 6 children (node.py:44-49)
        if (c < MZH_A) {
          *reinterpret_cast<uint32_t*>(&nb->nx[c]) = 0xFFFF0000u;  // N = 0, X = -1
          nb->R[c] = 0.0f;
          nb->P[c] = sm.pi[r * 8 + c];
          nb->W[c] = 0.0;
        }
        const int le = st.leafE[r], la = st.leafA[r], depth = st.depth[r];
        const float rew = sm.reward[r];
        double lmax = -__builtin_inf(), lmin = __builtin_inf();
        if (c == 0) {
          if (le == 0) {
            rb.X[la] = enew;
            rb.R[la] = rew;
          } else {
            tb[le].nx[la].X = (int16_t)enew;
            tb[le].R[la] = rew;
          }
          double v = (double)sm.value[r];
          int j = depth - 1;
          for (; j >= DC; --j) {  // beyond the LDS path cache (rare): update here from HBM
            const int slot = path[r * PL + j];
            const int e = slot >> 3, a = slot & 7;
            const double rw = (j == depth - 1) ? (double)rew : (double)tb[e].R[a];
            const double W = tb[e].W[a] + v;
            const int N = tb[e].nx[a].N + 1;
            tb[e].W[a] = W;
            tb[e].nx[a].N = (uint16_t)N;
            const double q = rw + disc * mzh_div(W, (double)N, inv[N]);
            lmax = q > lmax ? q : lmax;
            lmin = q < lmin ? q : lmin;
            v = rw + disc * v;
          }
          if (j == depth - 1 && j >= 0) {  // the leaf (its reward was just set)
            st.bval[r][j] = v;
            v = (double)rew + disc * v;
            --j;
          }
#pragma unroll 4
          for (; j >= 0; --j) {
            st.bval[r][j] = v;
            v = (double)st.pc[r][j].R + disc * v;
          }
          const double W = st.rootW[r] + v;
          const int N = st.rootN[r] + 1;
          st.rootW[r] = W;
          st.rootN[r] = N;
          const double q = 0.0 + disc * mzh_div(W, (double)N, inv[N]);  // root rwd = 0.0
          lmax = q > lmax ? q : lmax;
          lmin = q < lmin ? q : lmin;
        }
        __builtin_amdgcn_wave_barrier();
        const int jmax = depth < DC ? depth : DC;
        for (int j = c; j < jmax; j += 8) {
          const int slot = path[r * PL + j];
          const int e = slot >> 3, a = slot & 7;
          const MzhPathEnt pe = st.pc[r][j];
          const double rw = (j == depth - 1) ? (double)rew : (double)pe.R;
          const double W = pe.W + st.bval[r][j];
          const int N = pe.N + 1;
          if (e == 0) {
            rb.W[a] = W;
            rb.N[a] = N;
          } else {
            tb[e].W[a] = W;
            tb[e].nx[a].N = (uint16_t)N;
          }
          const double q = rw + disc * mzh_div(W, (double)N, inv[N]);
          lmax = q > lmax ? q : lmax;
          lmin = q < lmin ? q : lmin;
        }
        mzh_maxmin8d(lmax, lmin);
        if (c == 0) {
          const double mx = st.mm[r][0], mn = st.mm[r][1];
          mzh_mm_set(st.mm[r], lmax > mx ? lmax : mx, lmin < mn ? lmin : mn);
        }
      }
    }
    MZH_STAMP(22);
    __syncthreads();
    MZH_STAMP(23);
  }

  // ---------------- results (mcts.py:111-126, 154-176) ----------------
  if (tid < R * 8) {
    const int r = tid >> 3, c = tid & 7;
    if (r < nvalid && c == 0) {
      const int root = root0 + r;
      int vis[MZH_A];
      for (int a = 0; a < MZH_A; ++a) {
        vis[a] = st.root[r].N[a];
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
static size_t search_smem_bytes(int S, bool ohl) {
  size_t b = sizeof(MlpSmem<R>) + sizeof(SearchSmem<R>);
  b += sizeof(double) * 2 * (size_t)(S + 3);
  b += sizeof(uint16_t) * (size_t)((R * (S + 1) + 7) & ~7);
  if (ohl) b += sizeof(float) * MZH_A * MZH_F;
  return (b + 15) & ~(size_t)15;
}

static const size_t kLdsBytes = 163840;  // 160 KB per CU (gfx950)

// the minimum LDS a search launch needs at this R (one-hot columns left in HBM)
size_t mzh_search_smem_bytes(int R, int S) { return R == 32 ? search_smem_bytes<32>(S, false) : search_smem_bytes<16>(S, false); }

template <int R, bool REPLAY, bool OHL>
static hipError_t launch_search_t(const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const size_t smem = search_smem_bytes<R>(p.S, OHL);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mzh_search_kernel<R, REPLAY, OHL>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int grid = (p.B + R - 1) / R;
  hipLaunchKernelGGL((mzh_search_kernel<R, REPLAY, OHL>), dim3(grid), dim3(MZH_THREADS), smem, stream, net, p);
  return hipGetLastError();
}

hipError_t mzh_launch_search(int R, bool replay, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  if (R == 32) {
    if (replay) return launch_search_t<32, true, false>(net, p, stream);
    if (search_smem_bytes<32>(p.S, true) <= kLdsBytes) return launch_search_t<32, false, true>(net, p, stream);
    return launch_search_t<32, false, false>(net, p, stream);
  }
  return replay ? launch_search_t<16, true, false>(net, p, stream) : launch_search_t<16, false, false>(net, p, stream);
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

#ifdef MZH_STAMPS
// diagnostic build only: read and clear the accumulated phase stamps [8 waves][MZH_NSTAMP]
extern "C" int mzh_diag_stamps(unsigned long long* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(mzh_stamp_acc), sizeof(mzh_stamp_acc)) != hipSuccess) return -2;
  static unsigned long long zero[8][MZH_NSTAMP] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(mzh_stamp_acc), zero, sizeof(zero)) != hipSuccess) return -2;
  return 0;
}
#endif

hipError_t mzh_launch_infer(int R, bool recurrent, const MzhNet& net, const MzhInferParams& p, hipStream_t stream) {
  return R == 32 ? launch_infer_t<32>(recurrent, net, p, stream) : launch_infer_t<16>(recurrent, net, p, stream);
}
