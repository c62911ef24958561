// mzh_tree.h -- the search tree on the device: layout in HBM / LDS and the per-root select,
// expand/backup and result steps of the cooperative search kernels (mzh_search.hip,
// mzh_split.hip).  Each root is owned by one aligned 8-lane group (lane c = child slot c).
//
// Reference: MCTS/mcts.py:34-176 (run_mcts, generate_play_policy), MCTS/node.py:30-136
// (expand / backup / best_child / child_Q / child_U), MCTS/utils_mcts.py:1-16 (MinMaxStats).
#pragma once
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
// one child's selection operands except W, slot-major: N | X, reward and prior in one dwordx3
struct MzhSlot {
  MzhNX nx;
  float R;  // child reward (python float of an fp32 value, node.py:25)
  float P;  // child prior, fp32 (node.py:16)
};
struct __align__(128) MzhBlock {
  MzhSlot sl[6];  // 72 B
  double W[6];    // child summed value, fp64 (node.py:22)
  uint32_t pad[2];
};
static_assert(sizeof(MzhSlot) == 12, "slot layout");
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

template <int R, int DC_>
struct SearchSmem {
  static constexpr int DC = DC_;
  MzhRootBlk root[R];
  MzhPathEnt pc[R][DC + 1];  // entry DC: where the selection's stores of deeper levels land (never read)
  double rootW[R];
  double mm[R][4];  // MinMaxStats (maximum, minimum) + normaliser (max - min, RN(1/(max - min)))
  int rootN[R];
  int firstTie[R];
  int extra[R];
  int depth[R];
  int leafE[R];
  int leafA[R];
  int steps[R];
  int tie[R];  // the host-drawn index for the first 6-way tie (tie_idx)
  int lvl[2][MZH_WAVES];  // p.lockstep_levels: each wave's deepest selection, by selection parity
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

// MinMaxStats.normalize (utils_mcts.py:12-16) with den = max - min, dinv = RN(1/den).  The
// Markstein quotient needs a normal den (its reciprocal finite, the residual exact); `exact`
// (wave-uniform: some lane of the wave has a subnormal den -- only reachable from caller-given
// MinMaxStats bounds, never from fp32 network outputs) takes the IEEE division instead
__device__ __forceinline__ double mzh_normalize(double v, bool has, double mn, double den, double dinv, bool exact) {
  return has ? (exact ? (v - mn) / den : mzh_div(v - mn, den, dinv)) : v;
}
// whether any lane of the wave needs the exact normaliser (a non-zero subnormal max - min)
__device__ __forceinline__ bool mzh_need_exact(bool has, double den) {
  return __builtin_amdgcn_ballot_w64(has && !(den >= 2.2250738585072014e-308)) != 0;
}

// ucb = fl32(Q) + fl32(U) for one child (node.py:90-123); `tnp` = table[N_parent], inv[k] = RN(1/k)
// Branch-free: both reciprocals are read together (one ds_read2_b64) and the Q and U chains run side
// by side; for Nc = 0 the Q chain computes from inv[0] = inf and its result is discarded.
__device__ __forceinline__ float mzh_ucb(int Nc, double Wc, float Rc, double P64, bool p64_semantics, double tnp,
                                         double disc, bool has, double mn, double den, double dinv,
                                         const double* inv, bool exact) {
  const double i0 = inv[Nc], i1 = inv[Nc + 1];
  const double qn = mzh_normalize((double)Rc + disc * mzh_div(Wc, (double)Nc, i0), has, mn, den, dinv, exact);
  const float q32 = Nc > 0 ? (float)qn : 0.0f;
  const double w = mzh_div(tnp, (double)(Nc + 1), i1);
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
  const float m = mzh_max8_nonan(ucb);
  (void)c;  // lanes 6, 7 carry -inf, never the group maximum (the UCBs are finite)
  const unsigned long long bal = __builtin_amdgcn_ballot_w64(ucb == m);
  const unsigned mask = (unsigned)(bal >> (lane & ~7)) & 0x3Fu;
  const int cnt = __popc(mask);
  const int first = __ffs(mask) - 1;
  const bool six = (cnt == MZH_A) & (firstTie == 0);
  extra += ((cnt > 1) & !six) ? 1 : 0;
  firstTie |= six ? 1 : 0;
  return six ? tie : first;
}



// A root's search state between the tree steps, held in registers by every lane of its 8-lane group
// (all values group-uniform: every lane runs the value chain).  The LDS copy
// (SearchSmem) is read once before the first selection and written back once for the results.
struct MzhRootReg {
  double mmax, mmin, den, dinv;  // MinMaxStats + normaliser (mzh_mm_set)
  double rootW;
  int rootN, firstTie, extra, tie, steps;
  int depth, leafE, leafA;  // the current simulation's leaf (select -> backup)
  __device__ __forceinline__ void set_mm(double mx, double mn) {
    mmax = mx;
    mmin = mn;
    den = mx - mn;
    dinv = mx > mn ? 1.0 / (mx - mn) : 0.0;
  }
  template <int R, int DC>
  __device__ __forceinline__ void load(const SearchSmem<R, DC>& st, int r) {
    mmax = st.mm[r][0];
    mmin = st.mm[r][1];
    den = st.mm[r][2];
    dinv = st.mm[r][3];
    rootW = st.rootW[r];
    rootN = st.rootN[r];
    firstTie = st.firstTie[r];
    extra = st.extra[r];
    tie = st.tie[r];
    steps = st.steps[r];
    depth = st.depth[r];
    leafE = 0;
    leafA = 0;
  }
  template <int R, int DC>
  __device__ __forceinline__ void store(SearchSmem<R, DC>& st, int r) const {
    mzh_mm_set(st.mm[r], mmax, mmin);
    st.rootW[r] = rootW;
    st.rootN[r] = rootN;
    st.firstTie[r] = firstTie;
    st.extra[r] = extra;
    st.steps[r] = steps;
    st.depth[r] = depth;
  }
};

// Per-root steps over one workgroup's trees.  R roots (st / sm rows 0..R-1), DC path depths cached
// in LDS, `path` = [R][S + 1] selection slots.  SM: the MLP storage holding each root's row of the
// MLP input / output (x, act, pi, value, reward).
template <int R, int DC, bool REPLAY, class SM>
struct MzhTree {
  const MzhSearchParams& p;
  SearchSmem<R, DC>& st;
  SM& sm;
  uint16_t* path;
  const double* table;
  const double* inv;
  int root0, PL, lane;
  double disc;
  bool noised;

  // MMIN (the launch has caller-given MinMaxStats bounds): a wave with a root whose max - min is a
  // non-zero subnormal takes the exact-normaliser copy, chosen once per selection.  Without caller
  // bounds max - min is never subnormal (fresh bounds are +-inf; q values built from fp32 network
  // outputs are 0 or larger than 1e-70, so two distinct ones differ by far more than 2^-1022), and
  // the kernel carries only the Markstein copy.
  template <bool MMIN>
  __device__ __forceinline__ void select(const int r, const int c, const int s, MzhRootReg& rs) {
    if (MMIN && __builtin_expect(mzh_need_exact(rs.mmax > rs.mmin, rs.den), 0))
      select_impl<true>(r, c, s, rs);
    else
      select_impl<false>(r, c, s, rs);
  }

  template <bool EXACT>
  __device__ __forceinline__ void select_impl(const int r, const int c, const int s, MzhRootReg& rs) {
    const MzhBlock* tb = reinterpret_cast<const MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
    const double mmax = rs.mmax, mmin = rs.mmin, den = rs.den, dinv = rs.dinv;
    const bool has = mmax > mmin;
    constexpr bool exact = EXACT;
    int firstTie = rs.firstTie;
    int extra = rs.extra;
    const int tie = rs.tie;
    MZH_STAMP_DECL
#ifdef MZH_STAMPS
    asm volatile("" ::"v"(tie), "v"(dinv));
#endif
    MZH_STAMP(13);
    // level 0: the root block (LDS)
    int Nc = 0, Xc = -1;
    double Wc = 0.0;
    float Rc = 0.0f;
    float ucb;
    {  // all 8 slots of the root block are initialised (slots 6, 7: N = 0, X = -1, prior 0)
      const MzhRootBlk& rb = st.root[r];
      Nc = rb.N[c];
      Xc = rb.X[c];
      Wc = rb.W[c];
      Rc = rb.R[c];
      const float u = mzh_ucb(Nc, Wc, Rc, rb.P64[c], noised || p.np1, table[rs.rootN], disc, has, mmin, den, dinv, inv, exact);
      ucb = c < MZH_A ? u : -__builtin_inff();
    }
    int pick = mzh_group_pick(ucb, c, lane, tie, firstTie, extra);
    // every lane prefetches its own child's block (the selection's next level is one of
    // them): the block's cache lines are in flight while this level's UCB/argmax completes
    // (unconditional loads -- a lane without a child re-reads a valid block -- so the
    // compiler can count outstanding loads and wait only for the ones a level needs)
    int pf0 = *reinterpret_cast<const int*>(tb + (Xc >= 0 ? Xc : 0));
    // the packed (N | X << 16) word of the pick, taken over the group's DPP tree, moves the selection on
    int nx = mzh_group_take((Nc & 0xFFFF) | (Xc << 16), c == pick);
    int depth = 1, e = 0;

    // deeper levels: tree blocks in HBM (L2); lanes 6, 7 re-read slot 5 and act as
    // unexpanded, unvisited pads (N = 0, X = -1).  PIPE (16-root tiles): a level's block loads are
    // issued as soon as its block is known -- before the previous level's path stores, which then
    // run under their latency (the loads after the last level re-read the leaf's block, unused):
    // 4,096 roots -1.0%; the 32-root tile +0.4%, so it loads each level's block at the level's top
    constexpr bool PIPE = R == 16;
    const int cs = c < MZH_A ? c : MZH_A - 1;
    uint3 sv;   // N | X, R, P of this lane's slot: one dwordx3
    double Wl;  // W of this lane's slot
    auto issue = [&](int en, int ecur) {
      const MzhBlock* b = tb + (en >= 0 ? en : ecur);
      sv = *reinterpret_cast<const uint3*>(&b->sl[cs]);
      Wl = b->W[cs];
    };
    if (PIPE) issue(nx >> 16, 0);
    // the picking lane records the path entry and its own statistics
    if (c == pick) {
      path[r * PL] = (uint16_t)pick;
      st.pc[r][0] = MzhPathEnt{Wc, Rc, Nc};
    }
#ifdef MZH_STAMPS
    asm volatile("" ::"v"(nx), "v"(pf0));
#endif
    MZH_STAMP(14);
    MZH_LSTAMP_DECL
    while ((nx >> 16) >= 0) {
      e = nx >> 16;
      const int Np = nx & 0xFFFF;
      if (!PIPE) issue(e, e);
      const double tnp = table[Np];  // LDS: in flight beside the block loads
      int nxc = (int)sv.x;
      Rc = __uint_as_float(sv.y);
      Wc = Wl;
      const float Pc = __uint_as_float(sv.z);
      if (c >= MZH_A) nxc = (int)0xFFFF0000;
#ifdef MZH_STAMPS
      asm volatile("" ::"v"(nxc), "v"(Rc), "v"(Pc), "v"(Wc));
#endif
      MZH_LSTAMP(0);
      // retire the previous level's prefetch (older than this level's block loads, so no
      // extra wait) -- keeps it in flight inside the loop
      asm volatile("" ::"v"(pf0));
      const int xc = nxc >> 16;
      pf0 = *reinterpret_cast<const int*>(tb + (xc >= 0 ? xc : e));
      Nc = nxc & 0xFFFF;
      {
        const float u = mzh_ucb(Nc, Wc, Rc, (double)Pc, p.np1, tnp, disc, has, mmin, den, dinv, inv, exact);
        ucb = c < MZH_A ? u : -__builtin_inff();
      }
#ifdef MZH_STAMPS
      asm volatile("" ::"v"(ucb));
#endif
      MZH_LSTAMP(1);
      pick = mzh_group_pick(ucb, c, lane, tie, firstTie, extra);
#ifdef MZH_STAMPS
      asm volatile("" ::"v"(pick));
#endif
      MZH_LSTAMP(2);
      const int nxn = mzh_group_take(nxc, c == pick);
      if (PIPE) issue(nxn >> 16, e);
      if (c == pick) {  // two stores, no nested branch (levels past the cache land in entry DC)
        path[r * PL + depth] = (uint16_t)(e * 8 + pick);
        st.pc[r][depth < DC ? depth : DC] = MzhPathEnt{Wc, Rc, Nc};
      }
      nx = nxn;
      depth++;
#ifdef MZH_STAMPS
      asm volatile("" ::"v"(nx));
#endif
      MZH_LSTAMP(3);
      MZH_LSTAMP_COUNT();
    }
    MZH_LSTAMP_FLUSH(24);
    MZH_STAMP(15);
    rs.depth = depth;
    rs.leafE = e;
    rs.leafA = pick;
    rs.steps += depth;
    rs.firstTie = firstTie;
    rs.extra = extra;
    if (!REPLAY) {
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
      MZH_STAMP(31);
    }
    // the last level's prefetch is retired only here, so the latent loads above issue at the loop
    // exit instead of behind a wait for it (loads complete in issue order either way)
    asm volatile("" ::"v"(pf0));
  }

  // ---------------- expand bookkeeping + backup (node.py:30-70) of simulation s ----------------
  // Every lane of the root's group runs the value chain leaf -> root (two fp64 ops per level, the
  // only serial part) in registers, and keeps the values of the path depths j = c + 8k it updates
  // afterwards (no LDS hand-off, no wait between the levels); the 8 lanes then update the cached
  // path nodes in parallel and reduce the MinMaxStats candidates (max/min are exact and order-free).
  // val / rew: the new node's value and reward (every lane), pp: lane c's child prior
  __device__ __forceinline__ void backup(const int r, const int c, const int s, MzhRootReg& rs, float val, float rew,
                                         float pp) {
    MzhBlock* tb = reinterpret_cast<MzhBlock*>(p.tree) + (size_t)(root0 + r) * p.E;
    MzhRootBlk& rb = st.root[r];
    const int enew = s + 1;
    constexpr int NB = DC / 8;  // cached depths per lane
    // the reward snapshots of the cached depths, read before anything else (independent of the chain)
    float Rj[DC];
#pragma unroll
    for (int jj = 0; jj < DC; ++jj) Rj[jj] = st.pc[r][jj].R;
    MZH_STAMP_DECL
    if (!REPLAY) {
      // the new node's latent (read back when one of its children is expanded)
      const float* src = &sm.x[r * MZH_LD64 + c * 8];
      const floatx4 v0 = {src[0], src[1], src[2], src[3]}, v1 = {src[4], src[5], src[6], src[7]};
      {
        // the new node's latent is written through and not kept in the XCD's L2 (cache policy 16 = sc1):
        // at 32 roots a CU it would displace the tree blocks the next selections walk (the parent-latent
        // gather then reads it from the MALL).  8,192 roots -0.6%, 4,096 -1.1% (plain stores kept in L2;
        // the `nt` policy +1.3% / +0.7%, profiles/r05_coop_ab.json).  Workgroup-uniform base, the lane's
        // byte offset in a VGPR.
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t lr = mzh_rsrc(reinterpret_cast<floatx4*>(p.htree) + (size_t)root0 * p.E * 16);
        const int vo = ((r * p.E + enew) * 16 + c * 2) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), lr, vo, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v1), lr, vo + 16, 0, 16);
      }
    }
    MzhBlock* nb = tb + enew;  // the new expanded node's 6 children (node.py:44-49)
    if (c < MZH_A) {
      *reinterpret_cast<uint32_t*>(&nb->sl[c].nx) = 0xFFFF0000u;  // N = 0, X = -1
      nb->sl[c].R = 0.0f;
      nb->sl[c].P = pp;
      nb->W[c] = 0.0;
    }
    MZH_STAMP(16);
    const int le = rs.leafE, la = rs.leafA, depth = rs.depth;
    double lmax = -__builtin_inf(), lmin = __builtin_inf();
    if (c == 0) {
      if (le == 0) {
        rb.X[la] = enew;
        rb.R[la] = rew;
      } else {
        tb[le].sl[la].nx.X = (int16_t)enew;
        tb[le].sl[la].R = rew;
      }
    }
    double v = (double)val;
    int j = depth - 1;
    for (; j >= DC; --j) {  // beyond the LDS path cache (rare): lane j % 8 updates depth j from HBM
      const int slot = path[r * PL + j];
      const int e = slot >> 3, a = slot & 7;
      MzhBlock* eb = tb + e;
      const double rw = (j == depth - 1) ? (double)rew : (double)eb->sl[a].R;
      if (c == (j & 7)) {
        const double W = eb->W[a] + v;
        const int N = eb->sl[a].nx.N + 1;
        eb->W[a] = W;
        eb->sl[a].nx.N = (uint16_t)N;
        const double q = rw + disc * mzh_div(W, (double)N, inv[N]);
        lmax = q > lmax ? q : lmax;
        lmin = q < lmin ? q : lmin;
      }
      v = rw + disc * v;
    }
    // the cached depths j <= jtop: the fp64 chain in registers (the leaf takes its new reward); a
    // step above this lane's jtop keeps v, and steps above every active lane's jtop are skipped
    // (wave-uniform branch).  bv[k] = the value added at depth c + 8k.
    const int jtop = j;
    double bv[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) bv[k] = 0.0;
#pragma unroll
    for (int jj = DC - 1; jj >= 0; --jj) {
      if (!__any(jj <= jtop)) continue;
      if ((jj & 7) == c) bv[jj >> 3] = v;
      const double rw = jj == depth - 1 ? (double)rew : (double)Rj[jj];
      const double vn = rw + disc * v;
      v = jj <= jtop ? vn : v;
    }
    {  // the root (rwd = 0.0): every lane holds the same rootW
      const double W = rs.rootW + v;
      const int N = rs.rootN + 1;
      rs.rootW = W;
      const double q = 0.0 + disc * mzh_div(W, (double)N, inv[N]);
      lmax = q > lmax ? q : lmax;
      lmin = q < lmin ? q : lmin;
    }
    MZH_STAMP(17);
    const int jmax = depth < DC ? depth : DC;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int jp = c + 8 * k;
      if (jp < jmax) {
        const int slot = path[r * PL + jp];
        const int e = slot >> 3, a = slot & 7;
        const MzhPathEnt pe = st.pc[r][jp];
        const double rw = (jp == depth - 1) ? (double)rew : (double)pe.R;
        const double W = pe.W + bv[k];
        const int N = pe.N + 1;
        if (jp == 0) {  // the root's child (path entry 0 is the only one with e = 0)
          rb.W[a] = W;
          rb.N[a] = N;
        } else {
          tb[e].W[a] = W;
          tb[e].sl[a].nx.N = (uint16_t)N;
        }
        const double q = rw + disc * mzh_div(W, (double)N, inv[N]);
        lmax = q > lmax ? q : lmax;
        lmin = q < lmin ? q : lmin;
      }
    }
    MZH_STAMP(18);
    rs.rootN += 1;
    mzh_maxmin8d(lmax, lmin);
    rs.set_mm(lmax > rs.mmax ? lmax : rs.mmax, lmin < rs.mmin ? lmin : rs.mmin);
    MZH_STAMP(29);
  }

  // ---------------- results of root r (mcts.py:111-126, 154-176), one lane ----------------
  __device__ __forceinline__ void results(const int r) {
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
    if (p.latent && p.S > 0) {
      const int d = st.depth[r];
      for (int j = 0; j < d; ++j) p.latent[(size_t)root * PL + j] = path[r * PL + j] & 7;
      for (int j = d; j < PL; ++j) p.latent[(size_t)root * PL + j] = -1;
    }
    if (p.latent_len) p.latent_len[root] = p.S > 0 ? st.depth[r] : 0;
    if (p.pi || p.action) {
      double v[MZH_A];
      for (int a = 0; a < MZH_A; ++a) v[a] = (double)vis[a];
      if (p.temperature > 0.0) {
        double ex = 1.0 / p.temperature;
        ex = ex < 5.0 ? ex : 5.0;  // max(1.0, min(5.0, 1/T))
        ex = ex > 1.0 ? ex : 1.0;
        for (int a = 0; a < MZH_A; ++a) v[a] = mzh_pow(v[a], vis[a], ex, p.pow_table);
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
};
