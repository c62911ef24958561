// mzh_one.hip -- the latency path of the search: ONE root per workgroup, the network stationary on the CU.
//
// What it serves: MCTS.run_mcts as Muzero._play_game calls it -- one root, one search per environment step
// (Muzero.py:165-174, MCTS/mcts.py:34-126) -- and small root batches.  The cooperative kernel (mzh_search.hip)
// pads one root to a 16-row MFMA tile and streams the 0.49 MB of weights from L2 through the CU in every
// simulation; here a simulation is a chain of VALU dot products whose operands never leave the CU:
//   - the hidden layers' weight rows in registers for the whole launch (thread t < 256: unit t of
//     dynamic_net.0 and rwd_net.0; thread 256 + t: unit t of policy_net.0 and value_net.0), two waves per SIMD;
//   - the K = 256 output layers in LDS (MzhOneNet::l2, k-major, one ds_read_b128 per 4 k-steps);
//   - the root's tree (one 128-B MzhBlock per expanded node) in LDS; its latents in the engine's HBM workspace
//     (each lane re-reads only what it stored itself).
// Numerics are the oracle's (oracle/mzh_oracle.c): every dot product one k-ordered fmaf chain from 0 with the
// bias added after (bin 32 of a 33-bin head: four chains over k = g mod 4, ((p0 + p1) + (p2 + p3)) + bias),
// the one-hot action columns as the one non-zero step of that chain (acc + w: the zero steps add +-0 to a
// sum that is never -0), IEEE division in normalize_h_state, the heads through mzh_heads_row and the tree
// arithmetic through the helpers every search kernel shares (mzh_tree.h), so results equal the other kernels'
// bit for bit.
//
// Per simulation (mcts.py:71-109), with a workgroup barrier after each step:
//   dyn0 (waves 0-3) | dyn2 + normalize_h_state (wave 0) | rwd0 (waves 0-3) beside pol0 / val0 (waves 4-7) |
//   rwd2 / val2 bins 0-31 (wave 0), pol2 (wave 1), bin-32 chains (wave 2) |
//   heads + backup + the next selection + the parent-latent gather (wave 0; the root's 8-lane group)
#include "mzh_device.h"
#include "mzh_internal.h"
#include "mzh_tree.h"

namespace {
constexpr int kThreads = 512;  // 8 waves: two per SIMD, 256 registers each

struct MzhOneSmem {
  float obs[64];    // root observation (zero-padded)
  float xl[64];     // MLP input: the leaf's parent latent
  float hidD[256];  // dynamics hidden (root: representation hidden)
  float hraw[64];   // un-normalised latent (the reward head's input, networks.py:132-135)
  float xh[64];     // normalised latent (the prediction input)
  float hidR[256], hidP[256], hidV[256];
  float lrwd[40], lval[40], lpol[16];  // logits (natural order; mzh_heads_row strides MZH_LDSUP / MZH_LDPOL)
  float pi[8], value[1], reward[1];    // mzh_heads_row's STORE outputs (not used: STORE = false)
  int act;                             // the leaf's action (one-hot column of the next dyn0)
  int pad[3];
  MzhRootBlk root;                     // the root's 6 children (slots 6, 7 padding)
};

// LDS: the activations first (every access a small immediate offset from one lane base), then the LDS image
// of the output layers, the tree blocks, the UCB / reciprocal tables and the path
constexpr size_t kSmBytes = (sizeof(MzhOneSmem) + 127) & ~(size_t)127;
constexpr size_t kL2Bytes = (size_t)MZH_ONE_L2F4 * 16;
constexpr size_t kTreeOff = kSmBytes + kL2Bytes;

// y = sum_k x[k] * W[k][lane] over K = 256 as one k-ordered fmaf chain from 0 (oracle `linear`): W from the
// LDS image ([64 k4][NL lanes] float4), x from LDS (one broadcast ds_read_b128 per 4 k-steps)
template <int NL>
__device__ __forceinline__ float one_chain256(const float4* w, const float* x, int lane) {
  float acc = 0.0f;
#pragma unroll 2
  for (int k4 = 0; k4 < 64; ++k4) {
    const float4 wv = w[k4 * NL + lane];
    const float4 xv = reinterpret_cast<const float4*>(x)[k4];
    acc = __builtin_fmaf(xv.x, wv.x, acc);
    acc = __builtin_fmaf(xv.y, wv.y, acc);
    acc = __builtin_fmaf(xv.z, wv.z, acc);
    acc = __builtin_fmaf(xv.w, wv.w, acc);
  }
  return acc;
}

// K = 64 chain with the weight row in registers (x from LDS, broadcast)
__device__ __forceinline__ float one_chain64(const float* w, const float* x) {
  float acc = 0.0f;
#pragma unroll
  for (int k4 = 0; k4 < 16; ++k4) {
    const float4 xv = reinterpret_cast<const float4*>(x)[k4];
    acc = __builtin_fmaf(xv.x, w[4 * k4], acc);
    acc = __builtin_fmaf(xv.y, w[4 * k4 + 1], acc);
    acc = __builtin_fmaf(xv.z, w[4 * k4 + 2], acc);
    acc = __builtin_fmaf(xv.w, w[4 * k4 + 3], acc);
  }
  return acc;
}

__device__ __forceinline__ float one_relu(float v) { return v > 0.0f ? v : 0.0f; }

// normalize_h_state (networks.py:191-196) of the 64 units held one per lane of a full wave: min / max over
// the wave (exact, order-free), IEEE division as the oracle's normalize_h
__device__ __forceinline__ float one_normalize64(float h) {
  float mn = h, mx = h;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float a = __shfl_xor(mn, off), b = __shfl_xor(mx, off);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const float d = (mx - mn) + 9.999999939225290290778502821922302246094e-09f;
  return (h - mn) / d;
}
}  // namespace

size_t mzh_one_smem_bytes(int S) {
  size_t b = kTreeOff + (size_t)(S + 1) * sizeof(MzhBlock);  // tree blocks (block 0 = the root: unused)
  b += sizeof(double) * 2 * (size_t)(S + 3);                   // UCB table, RN(1/k)
  b += sizeof(uint16_t) * (size_t)(S + 1);                     // selection path
  return (b + 15) & ~(size_t)15;
}

// The root's 8-lane group (wave 0, lanes 0-7; lane c = child slot c) over the LDS tree.  The same operations,
// in the same order, as MzhTree (mzh_tree.h) -- node.py:53-123's arithmetic in fp64 with the shared helpers --
// only the storage differs: every block in LDS, the path a flat array.
struct MzhOneTree {
  const MzhSearchParams& p;
  MzhRootBlk& rb;
  MzhBlock* tb;
  uint16_t* path;
  const double* table;
  const double* inv;
  int lane;
  double disc;
  bool noised;

  template <bool EXACT>
  __device__ __forceinline__ void select_impl(const int c, MzhRootReg& rs) {
    const double mmax = rs.mmax, mmin = rs.mmin, den = rs.den, dinv = rs.dinv;
    const bool has = mmax > mmin;
    int firstTie = rs.firstTie, extra = rs.extra;
    const int tie = rs.tie;
    // level 0: the root block (all 8 slots initialised; slots 6, 7 never win)
    const int Nr = rb.N[c], Xr = rb.X[c];
    float ucb;
    {
      const float u = mzh_ucb(Nr, rb.W[c], rb.R[c], rb.P64[c], noised || p.np1, table[rs.rootN], disc, has, mmin, den,
                              dinv, inv, EXACT);
      ucb = c < MZH_A ? u : -__builtin_inff();
    }
    int pick = mzh_group_pick(ucb, c, lane, tie, firstTie, extra);
    int nx = mzh_group_take((Nr & 0xFFFF) | (Xr << 16), c == pick);
    if (c == pick) path[0] = (uint16_t)pick;
    int depth = 1, e = 0;
    const int cs = c < MZH_A ? c : MZH_A - 1;
    while ((nx >> 16) >= 0) {
      e = nx >> 16;
      const int Np = nx & 0xFFFF;
      const MzhBlock& b = tb[e];
      int nxc = *reinterpret_cast<const int*>(&b.sl[cs].nx);
      const float Rc = b.sl[cs].R, Pc = b.sl[cs].P;
      const double Wc = b.W[cs];
      if (c >= MZH_A) nxc = (int)0xFFFF0000;
      const int Nc = nxc & 0xFFFF;
      {
        const float u = mzh_ucb(Nc, Wc, Rc, (double)Pc, p.np1, table[Np], disc, has, mmin, den, dinv, inv, EXACT);
        ucb = c < MZH_A ? u : -__builtin_inff();
      }
      pick = mzh_group_pick(ucb, c, lane, tie, firstTie, extra);
      nx = mzh_group_take(nxc, c == pick);
      if (c == pick) path[depth] = (uint16_t)(e * 8 + pick);
      depth++;
    }
    rs.depth = depth;
    rs.leafE = e;
    rs.leafA = pick;
    rs.steps += depth;
    rs.firstTie = firstTie;
    rs.extra = extra;
  }

  // MMIN (caller-given MinMaxStats bounds): the exact normaliser when max - min is a non-zero subnormal
  template <bool MMIN>
  __device__ __forceinline__ void select(const int c, MzhRootReg& rs) {
    if (MMIN && __builtin_expect(mzh_need_exact(rs.mmax > rs.mmin, rs.den), 0))
      select_impl<true>(c, rs);
    else
      select_impl<false>(c, rs);
  }

  // expand bookkeeping + backup (node.py:30-70) of simulation s: the new node's children, the leaf's link and
  // reward, then the fp64 value chain leaf -> root on every lane, lane j % 8 updating path depth j
  __device__ __forceinline__ void backup(const int c, const int s, MzhRootReg& rs, float val, float rew, float pp) {
    const int enew = s + 1;
    if (c < MZH_A) {
      MzhSlot& sl = tb[enew].sl[c];
      *reinterpret_cast<uint32_t*>(&sl.nx) = 0xFFFF0000u;  // N = 0, X = -1
      sl.R = 0.0f;
      sl.P = pp;
      tb[enew].W[c] = 0.0;
    }
    const int le = rs.leafE, la = rs.leafA, depth = rs.depth;
    if (c == 0) {
      if (le == 0) {
        rb.X[la] = enew;
        rb.R[la] = rew;
      } else {
        tb[le].sl[la].nx.X = (int16_t)enew;
        tb[le].sl[la].R = rew;
      }
    }
    double lmax = -__builtin_inf(), lmin = __builtin_inf();
    double v = (double)val;
    for (int j = depth - 1; j >= 0; --j) {
      const int ent = path[j];
      const int e = j == 0 ? 0 : ent >> 3, a = j == 0 ? ent : ent & 7;
      double W;
      int N;
      float Rn;
      if (j == 0) {
        W = rb.W[a];
        N = rb.N[a];
        Rn = rb.R[a];
      } else {
        W = tb[e].W[a];
        N = tb[e].sl[a].nx.N;
        Rn = tb[e].sl[a].R;
      }
      const double rw = j == depth - 1 ? (double)rew : (double)Rn;
      if (c == (j & 7)) {
        const double Wn = W + v;
        const int Nn = N + 1;
        if (j == 0) {
          rb.W[a] = Wn;
          rb.N[a] = Nn;
        } else {
          tb[e].W[a] = Wn;
          tb[e].sl[a].nx.N = (uint16_t)Nn;
        }
        const double q = rw + disc * mzh_div(Wn, (double)Nn, inv[Nn]);
        lmax = q > lmax ? q : lmax;
        lmin = q < lmin ? q : lmin;
      }
      v = rw + disc * v;
    }
    {  // the root (rwd = 0.0): every lane holds the same rootW
      const double W = rs.rootW + v;
      const int N = rs.rootN + 1;
      rs.rootW = W;
      const double q = 0.0 + disc * mzh_div(W, (double)N, inv[N]);
      lmax = q > lmax ? q : lmax;
      lmin = q < lmin ? q : lmin;
    }
    rs.rootN += 1;
    mzh_maxmin8d(lmax, lmin);
    rs.set_mm(lmax > rs.mmax ? lmax : rs.mmax, lmin < rs.mmin ? lmin : rs.mmin);
  }

  // results of root r (mcts.py:111-126, 154-176): MzhTree::results from the registers / LDS, one lane
  __device__ __forceinline__ void results(const int root, const MzhRootReg& rs) {
    const int PL = p.S + 1;
    int vis[MZH_A];
    for (int a = 0; a < MZH_A; ++a) {
      vis[a] = rb.N[a];
      p.visits[(size_t)root * MZH_A + a] = vis[a];
    }
    if (p.root_q) p.root_q[root] = rs.rootN == 0 ? 0.0 : rs.rootW / (double)rs.rootN;
    if (p.minmax_out) {
      p.minmax_out[2 * root] = rs.mmax;
      p.minmax_out[2 * root + 1] = rs.mmin;
    }
    if (p.extra_ties) p.extra_ties[root] = rs.extra;
    if (p.sel_steps) p.sel_steps[root] = rs.steps;
    const int d = p.S > 0 ? rs.depth : 0;
    if (p.latent && p.S > 0) {
      for (int j = 0; j < d; ++j) p.latent[(size_t)root * PL + j] = path[j] & 7;
      for (int j = d; j < PL; ++j) p.latent[(size_t)root * PL + j] = -1;
    }
    if (p.latent_len) p.latent_len[root] = d;
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

// a value the compiler must treat as new at this point: per-lane index arithmetic derived from it is redone
// inside the loop instead of being hoisted out of the root / simulation loops and kept live (with 134 weight
// registers per lane those hoisted 64-bit addresses were what spilled)
__device__ __forceinline__ int one_fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <bool SUP33, bool MMIN>
__global__ __launch_bounds__(512, 2) void mzh_search_one_kernel(MzhNet net, MzhOneNet on, MzhSearchParams p) {
  extern __shared__ __align__(128) unsigned char smem_raw[];
  MzhOneSmem& sm = *reinterpret_cast<MzhOneSmem*>(smem_raw);
  float4* l2 = reinterpret_cast<float4*>(smem_raw + kSmBytes);
  const float* l2f = reinterpret_cast<const float*>(smem_raw + kSmBytes);
  MzhBlock* tb = reinterpret_cast<MzhBlock*>(smem_raw + kTreeOff);
  const int S = p.S;
  double* table = reinterpret_cast<double*>(tb + (S + 1));
  double* inv = table + (S + 3);  // inv[k] = RN(1/k), k <= S + 2
  uint16_t* path = reinterpret_cast<uint16_t*>(inv + (S + 3));

  const int t = threadIdx.x, wave = t >> 6;
  const bool A = t < 256;  // waves 0-3: dynamic_net.0 / rwd_net.0 rows; waves 4-7: policy_net.0 / value_net.0
  const __amdgpu_buffer_rsrc_t wres = mzh_rsrc(on.l1);  // every weight array lies in the one packed blob
  const int wbase = 0;
  // the hidden layers' weight rows of unit t % 256, in registers for the whole launch
  float w1[64], w2[64], woh[6];
  float b1a, b1b;
  {
    const int n = t & 255, k0 = A ? 0 : 32;
#pragma unroll
    for (int k4 = 0; k4 < 16; ++k4) {
      const floatx4 a = mzh_ld4(wres, 16 * n, wbase + ((k0 + k4) * 256) * 16);
      const floatx4 b = mzh_ld4(wres, 16 * n, wbase + ((k0 + 16 + k4) * 256) * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w1[4 * k4 + i] = a[i];
        w2[4 * k4 + i] = b[i];
      }
    }
    const floatx4 o0 = mzh_ld4(wres, 16 * n, 64 * 256 * 16), o1 = mzh_ld4(wres, 16 * n, 65 * 256 * 16);
    woh[0] = o0[0]; woh[1] = o0[1]; woh[2] = o0[2]; woh[3] = o0[3]; woh[4] = o1[0]; woh[5] = o1[1];
    const float4 bb = on.b1[n];
    b1a = A ? bb.x : bb.z;
    b1b = A ? bb.y : bb.w;
  }
  const __amdgpu_buffer_rsrc_t l2res = mzh_rsrc(on.l2), r2res = mzh_rsrc(on.rep2);
  for (int i = t; i < MZH_ONE_L2F4; i += kThreads)
    *reinterpret_cast<floatx4*>(&l2[i]) = mzh_ld4(l2res, 16 * i, 0);
  for (int i = t; i < S + 3; i += kThreads) {
    table[i] = i < S + 2 ? p.table[i] : 0.0;
    inv[i] = 1.0 / (double)i;  // IEEE division: correctly rounded
  }
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;
  const int support = net.support;
  __syncthreads();

  for (int r = blockIdx.x; r < p.B; r += gridDim.x) {
    // this root's latents [E][64] in the engine's workspace: lane j stores and re-reads element j
    const __amdgpu_buffer_rsrc_t lres = mzh_rsrc(p.htree + (size_t)r * p.E * MZH_H);
    const int tr = one_fresh(t), lane = tr & 63, n = tr & 255, c = lane & 7;
    const bool grp = wave == 0 && lane < 8;  // the root's 8-lane group (tree phases)
    MzhOneTree tree{p, sm.root, tb, path, table, inv, lane, disc, noised};
    // ---------------- root: initial_inference (mcts.py:49-50, networks.py:71-94) ----------------
    if (t < 64) sm.obs[lane] = lane < p.in_dim ? p.obs[(size_t)r * p.in_dim + lane] : 0.0f;
    // representation_net.2 into the dynamic_net.2 region (reloaded below, before the first simulation)
#pragma unroll
    for (int i = 0; i < 8; ++i)
      *reinterpret_cast<floatx4*>(&l2[MZH_ONE_D2 + tr + 512 * i]) = mzh_ld4(r2res, 16 * tr, 16 * 512 * i);
    __syncthreads();
    if (A) {  // representation_net.0 (K = 3N), unit n, weights k-major from L2
      const __amdgpu_buffer_rsrc_t r0 = mzh_rsrc(on.rep0);
      float acc = 0.0f;
      for (int k = 0; k < p.in_dim; ++k) acc = __builtin_fmaf(sm.obs[k], mzh_ld1(r0, 4 * n, k * 1024), acc);
      sm.hidD[n] = one_relu(acc + on.rep0b[n]);
    }
    __syncthreads();
    if (wave == 0) {  // representation_net.2 + normalize_h_state
      const float h = one_chain256<64>(l2 + MZH_ONE_D2, sm.hidD, lane) + on.rep2b[lane];
      const float hn = one_normalize64(h);
      sm.xh[lane] = hn;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hn), lres, 4 * lane, 0, 0);  // node 0's latent
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i)
      *reinterpret_cast<floatx4*>(&l2[MZH_ONE_D2 + tr + 512 * i]) =
          mzh_ld4(l2res, 16 * tr, 16 * (MZH_ONE_D2 + 512 * i));
    if (!A) {  // prediction hidden layers
      float ap = 0.0f, av = 0.0f;
#pragma unroll
      for (int k4 = 0; k4 < 16; ++k4) {
        const float4 xv = reinterpret_cast<const float4*>(sm.xh)[k4];
        ap = __builtin_fmaf(xv.x, w1[4 * k4], ap);
        av = __builtin_fmaf(xv.x, w2[4 * k4], av);
        ap = __builtin_fmaf(xv.y, w1[4 * k4 + 1], ap);
        av = __builtin_fmaf(xv.y, w2[4 * k4 + 1], av);
        ap = __builtin_fmaf(xv.z, w1[4 * k4 + 2], ap);
        av = __builtin_fmaf(xv.z, w2[4 * k4 + 2], av);
        ap = __builtin_fmaf(xv.w, w1[4 * k4 + 3], ap);
        av = __builtin_fmaf(xv.w, w2[4 * k4 + 3], av);
      }
      sm.hidP[n] = one_relu(ap + b1a);
      sm.hidV[n] = one_relu(av + b1b);
    }
    __syncthreads();
    if (wave == 0 && lane >= 32) {  // value_net.2 bins 0-31
      const float acc = one_chain256<64>(l2 + MZH_ONE_A2, sm.hidV, lane);
      sm.lval[lane - 32] = acc + l2f[MZH_ONE_B2 * 4 + 64 + lane];
    } else if (wave == 1 && lane < 8) {  // policy_net.2
      const float acc = one_chain256<8>(l2 + MZH_ONE_P2, sm.hidP, lane);
      if (lane < MZH_A) sm.lpol[lane] = acc + l2f[MZH_ONE_B2 * 4 + 128 + lane];
    } else if (SUP33 && wave == 2 && lane >= 4 && lane < 8) {  // value bin 32: four chains over k = g mod 4
      const int g = lane & 3;
      const float* cw = l2f + MZH_ONE_C32 * 4 + lane;
      float acc = 0.0f;
#pragma unroll 8
      for (int i = 0; i < 64; ++i) acc = __builtin_fmaf(sm.hidV[g + 4 * i], cw[8 * i], acc);
      acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0xB1, 0xF, 0xF, true));  // p0+p1 | p2+p3
      acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x4E, 0xF, 0xF, true));
      if (lane == 4) sm.lval[32] = acc + l2f[MZH_ONE_B2 * 4 + 137];
    }
    __syncthreads();
    MzhRootReg rs;
    if (grp) {
      const MzhHeadOut ho = mzh_heads_row<1, SUP33 ? 33 : 0, false, false>(sm, net, 0, c, support, false);
      // root.expand(prior, h, 0) with optional Dirichlet mixing (mcts.py:57-69, 132-152)
      MzhRootBlk& rb = sm.root;
      const float pr = c < MZH_A ? ho.pp : 0.0f;
      rb.N[c] = 0;
      rb.X[c] = -1;
      rb.R[c] = 0.0f;
      rb.W[c] = 0.0;
      double v = (double)pr;
      if (noised && c < MZH_A) {
        const float scaled = (float)(1.0 - p.eps) * pr;  // (1-eps) * prob, float32 array
        v = (double)scaled + p.eps * p.noise[(size_t)r * MZH_A + c];
      }
      rb.P64[c] = v;
      double mx = -__builtin_inf(), mn = __builtin_inf();
      if (p.minmax_in) {
        mx = p.minmax_in[2 * r];
        mn = p.minmax_in[2 * r + 1];
      }
      rs.set_mm(mx, mn);
      rs.rootW = 0.0;
      rs.rootN = 0;
      rs.firstTie = 0;
      rs.extra = 0;
      rs.tie = p.tie_idx ? p.tie_idx[r] : 0;
      rs.steps = 0;
      rs.depth = 0;
      rs.leafE = 0;
      rs.leafA = 0;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if (S > 0) tree.template select<MMIN>(c, rs);
    }
    int lsum = 0;  // p.lockstep_levels: this root's selection levels below the root, summed
    if (wave == 0 && S > 0) {
      const int e = __shfl(rs.leafE, 0), a = __shfl(rs.leafA, 0);
      lsum += __shfl(rs.depth, 0) - 1;
      // the leaf's parent latent (mcts.py:89-92), stored by this lane
      sm.xl[lane] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lres, 4 * lane, 4 * MZH_H * e, 0));
      if (lane == 0) sm.act = a;
    }
    __syncthreads();
    for (int s = 0; s < S; ++s) {
      const int ts = one_fresh(t), ls = ts & 63, ns = ts & 255;
      // ---------------- expand via the network (mcts.py:88-106, networks.py:96-150) ----------------
      if (A) {  // dynamic_net.0: 64 latent steps, the one-hot column, bias, ReLU
        float acc = one_chain64(w1, sm.xl);
        const int a = sm.act;
        const float wa = a == 0 ? woh[0] : a == 1 ? woh[1] : a == 2 ? woh[2] : a == 3 ? woh[3] : a == 4 ? woh[4] : woh[5];
        acc = acc + wa;
        sm.hidD[ns] = one_relu(acc + b1a);
      }
      __syncthreads();
      if (wave == 0) {  // dynamic_net.2 (K = 256), then normalize_h_state
        const float hr = one_chain256<64>(l2 + MZH_ONE_D2, sm.hidD, ls) + l2f[MZH_ONE_B2 * 4 + ls];
        sm.hraw[ls] = hr;
        const float hn = one_normalize64(hr);
        sm.xh[ls] = hn;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hn), lres, 4 * ls, 4 * MZH_H * (s + 1), 0);
      }
      __syncthreads();
      if (A) {  // rwd_net.0 on the un-normalised latent
        sm.hidR[ns] = one_relu(one_chain64(w2, sm.hraw) + b1b);
      } else {  // policy_net.0 / value_net.0 on the normalised latent
        float ap = 0.0f, av = 0.0f;
#pragma unroll
        for (int k4 = 0; k4 < 16; ++k4) {
          const float4 xv = reinterpret_cast<const float4*>(sm.xh)[k4];
          ap = __builtin_fmaf(xv.x, w1[4 * k4], ap);
          av = __builtin_fmaf(xv.x, w2[4 * k4], av);
          ap = __builtin_fmaf(xv.y, w1[4 * k4 + 1], ap);
          av = __builtin_fmaf(xv.y, w2[4 * k4 + 1], av);
          ap = __builtin_fmaf(xv.z, w1[4 * k4 + 2], ap);
          av = __builtin_fmaf(xv.z, w2[4 * k4 + 2], av);
          ap = __builtin_fmaf(xv.w, w1[4 * k4 + 3], ap);
          av = __builtin_fmaf(xv.w, w2[4 * k4 + 3], av);
        }
        sm.hidP[ns] = one_relu(ap + b1a);
        sm.hidV[ns] = one_relu(av + b1b);
      }
      __syncthreads();
      if (wave == 0) {  // rwd_net.2 bins 0-31 (lanes 0-31) | value_net.2 bins 0-31 (lanes 32-63)
        const float acc = one_chain256<64>(l2 + MZH_ONE_A2, ls < 32 ? sm.hidR : sm.hidV, ls);
        const float y = acc + l2f[MZH_ONE_B2 * 4 + 64 + ls];
        if (ls < 32)
          sm.lrwd[ls] = y;
        else
          sm.lval[ls - 32] = y;
      } else if (wave == 1 && ls < 8) {  // policy_net.2
        const float acc = one_chain256<8>(l2 + MZH_ONE_P2, sm.hidP, ls);
        if (ls < MZH_A) sm.lpol[ls] = acc + l2f[MZH_ONE_B2 * 4 + 128 + ls];
      } else if (SUP33 && wave == 2 && ls < 8) {  // bin 32 of both heads: lane 4h + g runs chain g of head h
        const int g = ls & 3;
        const float* hid = ls < 4 ? sm.hidR : sm.hidV;
        const float* cw = l2f + MZH_ONE_C32 * 4 + ls;
        float acc = 0.0f;
#pragma unroll 8
        for (int i = 0; i < 64; ++i) acc = __builtin_fmaf(hid[g + 4 * i], cw[8 * i], acc);
        acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0xB1, 0xF, 0xF, true));
        acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x4E, 0xF, 0xF, true));
        if (ls == 0) sm.lrwd[32] = acc + l2f[MZH_ONE_B2 * 4 + 136];
        if (ls == 4) sm.lval[32] = acc + l2f[MZH_ONE_B2 * 4 + 137];
      }
      __syncthreads();
      // ---------------- heads, backup (node.py:53-70), the next selection ----------------
      if (grp) {
        const MzhHeadOut ho = mzh_heads_row<1, SUP33 ? 33 : 0, false, false>(sm, net, 0, ls & 7, support, true);
        tree.backup(ls & 7, s, rs, ho.value, ho.reward, ho.pp);
        if (s + 1 < S) {
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
          __builtin_amdgcn_wave_barrier();
          tree.template select<MMIN>(ls & 7, rs);
        }
      }
      if (wave == 0 && s + 1 < S) {
        const int e = __shfl(rs.leafE, 0), a = __shfl(rs.leafA, 0);
        lsum += __shfl(rs.depth, 0) - 1;
        sm.xl[ls] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lres, 4 * ls, 4 * MZH_H * e, 0));
        if (ls == 0) sm.act = a;
      }
      __syncthreads();
    }
    // ---------------- results (mcts.py:111-126, 154-176) ----------------
    if (wave == 0 && lane == 0) {
      tree.results(r, rs);
      if (p.lockstep_levels) p.lockstep_levels[r] = lsum;
    }
    __syncthreads();  // the next root reuses the LDS tree and activations
  }
}

template <bool SUP33, bool MMIN>
static hipError_t launch_one_t(const MzhNet& net, const MzhOneNet& on, const MzhSearchParams& p, int grid,
                               hipStream_t stream) {
  const size_t smem = mzh_one_smem_bytes(p.S);
  const void* fn = reinterpret_cast<const void*>(&mzh_search_one_kernel<SUP33, MMIN>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((mzh_search_one_kernel<SUP33, MMIN>), dim3(grid), dim3(kThreads), smem, stream, net, on, p);
  return hipGetLastError();
}

hipError_t mzh_launch_one(const MzhSearchPlan& pl, const MzhNet& net, const MzhOneNet& on, const MzhSearchParams& p,
                          hipStream_t stream) {
  const int grid = pl.grid;  // min(B, 256): one round of workgroups, each persistent over its roots
  if (pl.sup33) return pl.mmin ? launch_one_t<true, true>(net, on, p, grid, stream) : launch_one_t<true, false>(net, on, p, grid, stream);
  return pl.mmin ? launch_one_t<false, true>(net, on, p, grid, stream) : launch_one_t<false, false>(net, on, p, grid, stream);
}
