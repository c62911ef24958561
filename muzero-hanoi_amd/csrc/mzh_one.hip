// mzh_one.hip -- the latency path of the search: ONE root per workgroup, the network stationary on the CU.
//
// What it serves: MCTS.run_mcts as Muzero._play_game calls it -- one root, one search per environment step
// (Muzero.py:165-174, MCTS/mcts.py:34-126) -- and small root batches.  The cooperative kernel (mzh_search.hip)
// pads one root to a 16-row MFMA tile and streams the 0.49 MB of weights from L2 through the CU in every
// simulation; here a simulation is a chain of VALU dot products whose operands never leave the CU, one
// v_fmac_f32_dpp (row_newbcast: the activation from lane j of the lane's own 16-lane row) per k-step:
//   - the hidden layers' weight rows in registers for the whole launch (thread t < 256: unit t of
//     dynamic_net.0 and rwd_net.0; thread 256 + t: unit t of policy_net.0 and value_net.0), two waves per SIMD;
//   - the K = 256 output layers in LDS (MzhOneNet::l2, k-major, one ds_read_b128 per 4 k-steps);
//   - the root's tree (one 128-B MzhBlock per expanded node) in LDS; its latents in LDS too where they fit
//     (LATL, n_sims up to ~36), else in the engine's HBM workspace (each lane re-reads only what it stored).
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

// Activations in the "row layouts" the chains read (one_rows): a K = 256 vector as T[16][20] (element 16v + j at
// T[j][v]: lane l finds x[16v + (l & 15)], v = 0..15, in four ds_read_b128; the stride of 20 floats puts the 16 rows'
// reads in distinct banks), a K = 64 vector as T[16][4]; the bin-32 chains' copies Q[4][68] (unit g + 4i at Q[g][i]).
struct MzhOneSmem {
  float obs[64];                        // root observation (zero-padded)
  float xlT[64];                        // MLP input: the leaf's parent latent (T64)
  float hidDT[320];                     // dynamics (root: representation) hidden (T256)
  float hrawT[64];                      // un-normalised latent, the reward head's input (networks.py:132-135) (T64)
  float xhT[64];                        // normalised latent, the prediction input (T64)
  float hidRT[320], hidPT[320], hidVT[320];  // reward / policy / value hidden (T256)
  float hidRQ[272], hidVQ[272];         // reward / value hidden for bin 32's chains (Q)
  float lrwd[40], lval[40], lpol[16];   // logits (natural order)
  int act;                              // the leaf's action (one-hot column of the next dyn0)
  int pad[3];
  MzhRootBlk root;                      // the root's 6 children (slots 6, 7 padding)
  MzhRootReg rsv;                       // the root's search state between tree phases (not live in registers
                                        // across the MLP: every register there holds weights or chain operands)
};
__device__ __forceinline__ int one_t256(int n) { return (n & 15) * 20 + (n >> 4); }
__device__ __forceinline__ int one_t64(int j) { return (j & 15) * 4 + (j >> 4); }
__device__ __forceinline__ int one_q(int n) { return (n & 3) * 68 + (n >> 2); }

constexpr size_t kSmBytes = (sizeof(MzhOneSmem) + 127) & ~(size_t)127;
constexpr size_t kL2Bytes = (size_t)MZH_ONE_L2F4 * 16;
constexpr size_t kTreeOff = kSmBytes + kL2Bytes;

// y = sum_k x[k] * W[k][lane] over K = 256 as one k-ordered fmaf chain from 0 (oracle `linear`): W from the
// LDS image ([64 k4][NL lanes] float4), x from LDS (one broadcast ds_read_b128 per 4 k-steps)
// 16 k-steps of a dot-product chain, acc = fmaf(x[16v + j], w[j], acc) for j = 0..15 in order: x comes from
// lane j of the lane's own 16-lane row (DPP row_newbcast:j -- every row holds x[16v .. 16v + 15], one per lane), so
// a k-step is ONE v_fmac_f32 with no LDS read for the broadcast operand.  Wait states the compiler cannot see
// inside the asm: 2 between a VALU write of xv and its DPP read, 5 between a VALU write of EXEC and a DPP op --
// s_nop 4 before a chain's first block (it may follow a branch), s_nop 1 before the others.
#define MZH_FMAC(j, wi) "v_fmac_f32_dpp %0, %1, %" #wi " row_newbcast:" #j " row_mask:0xf bank_mask:0xf\n\t"
#define MZH_FMA16(NOP)                                                                                            \
  asm(NOP MZH_FMAC(0, 2) MZH_FMAC(1, 3) MZH_FMAC(2, 4) MZH_FMAC(3, 5) MZH_FMAC(4, 6) MZH_FMAC(5, 7) MZH_FMAC(6, 8)      \
          MZH_FMAC(7, 9) MZH_FMAC(8, 10) MZH_FMAC(9, 11) MZH_FMAC(10, 12) MZH_FMAC(11, 13) MZH_FMAC(12, 14)          \
              MZH_FMAC(13, 15) MZH_FMAC(14, 16) MZH_FMAC(15, 17)                                                    \
      : "+v"(acc)                                                                                                   \
      : "v"(xv), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]), \
        "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15]))
template <bool FIRST = false>
__device__ __forceinline__ void one_fma16(float& acc, float xv, const float* w) {
  if constexpr (FIRST)
    MZH_FMA16("s_nop 4\n\t");
  else
    MZH_FMA16("s_nop 1\n\t");
}
#undef MZH_FMA16
#undef MZH_FMAC

// the row layout of a K-vector for one_fma16: lane l holds x[16v + (l & 15)] in xr[v], read from T256 / T64
template <int NV>
__device__ __forceinline__ void one_rows(float* xr, const float* xT, int lane) {
  const float4* r = reinterpret_cast<const float4*>(xT + (lane & 15) * (NV == 16 ? 20 : 4));
#pragma unroll
  for (int m = 0; m < NV / 4; ++m) {
    const float4 q = r[m];
    xr[4 * m] = q.x;
    xr[4 * m + 1] = q.y;
    xr[4 * m + 2] = q.z;
    xr[4 * m + 3] = q.w;
  }
}

// y = sum_k x[k] * W[k][wl] over K = 256 as one k-ordered fmaf chain from 0 (oracle `linear`): W from the
// LDS image ([64 k4][NL lanes] float4, kept 8 reads ahead), x in the row layout (one_rows).  Every lane of a
// 16-lane row the DPP broadcast reads from must be active: a disabled source lane disables the FMA.
template <int NL>
__device__ __forceinline__ float one_chain256(const float4* w, const float* x, int wl, int lane) {
  float xr[16];
  one_rows<16>(xr, x, lane);
  constexpr int D = 8;
  // one base address register, every read an immediate offset from it (laundered: left to itself the compiler
  // folds the region offset into per-read constants beyond the 64 KiB offset range and rematerialises them)
  typedef __attribute__((address_space(3))) const floatx4 LdsF4;
  LdsF4* wp = (LdsF4*)(w + wl);
  asm volatile("" : "+v"(wp));
  floatx4 wb[D];
#pragma unroll
  for (int i = 0; i < D; ++i) wb[i] = wp[i * NL];
  // every x read and the first D weight reads issue before the first FMA (LDS completes in issue order: a
  // block then waits only for its own weights, not for reads issued after them)
  __builtin_amdgcn_sched_barrier(0);
  float acc = 0.0f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    float ww[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const floatx4 q = wb[(4 * v + i) % D];
      ww[4 * i] = q[0];
      ww[4 * i + 1] = q[1];
      ww[4 * i + 2] = q[2];
      ww[4 * i + 3] = q[3];
    }
    if (v == 0)
      one_fma16<true>(acc, xr[v], ww);
    else
      one_fma16(acc, xr[v], ww);
    // refill the block's slots with the weights D / 4 blocks ahead, after its FMAs (no copy of the slots)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k4 = 4 * v + i;
      if (k4 + D < 64) wb[k4 % D] = wp[(k4 + D) * NL];
    }
  }
  return acc;
}

// K = 64 chain with the weight row in registers, x in the row layout
__device__ __forceinline__ float one_chain64(const float* w, const float* x, int lane) {
  float xr[4];
  one_rows<4>(xr, x, lane);
  float acc = 0.0f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    if (v == 0)
      one_fma16<true>(acc, xr[v], w);
    else
      one_fma16(acc, xr[v], w + 16 * v);
  }
  return acc;
}

__device__ __forceinline__ float one_relu(float v) { return v > 0.0f ? v : 0.0f; }

// bin 32 of a 33-bin head, chain g (oracle linear_head): fmaf over hidden units k = g, g + 4, ..., g + 252 in order,
// x from Q[g] and the weights [64] (this lane's MZH_ONE_C32 row), as float4 runs kept D reads ahead (the chain
// waits only for its own operands; fully unrolled without the ring, the scheduler hoists all 32 reads and the
// 128 registers they take evict the weight rows the kernel keeps resident).
__device__ __forceinline__ float one_chain_bin32(const float* q, const float* w) {
  typedef __attribute__((address_space(3))) const floatx4 LdsF4;
  LdsF4* xq = (LdsF4*)q;
  LdsF4* wq = (LdsF4*)w;
  asm volatile("" : "+v"(xq), "+v"(wq));
  constexpr int D = 4;
  floatx4 xb[D], wb[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    xb[i] = xq[i];
    wb[i] = wq[i];
  }
  float acc = 0.0f;
  // rolled by D (ring slots static in the body); the last trip's refills read the 4 float4 past the run, inside
  // the LDS image (Q's padding, the next row / the bias block) and unused
#pragma unroll 1
  for (int m = 0; m < 16; m += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const floatx4 xv = xb[i], wv = wb[i];
      acc = __builtin_fmaf(xv[0], wv[0], acc);
      acc = __builtin_fmaf(xv[1], wv[1], acc);
      acc = __builtin_fmaf(xv[2], wv[2], acc);
      acc = __builtin_fmaf(xv[3], wv[3], acc);
      xb[i] = xq[m + D + i];
      wb[i] = wq[m + D + i];
    }
  }
  return acc;
}

// The heads (networks.py:83,109,152-189) of mzh_heads_row with its two 33-bin heads on two 8-lane groups
// instead of side by side on one: lanes 0-7 the value head (and the policy softmax), lanes 8-15 the reward head
// (and a copy of the policy softmax), so one instruction stream serves both.  Every operation and summation
// order of a head is mzh_heads_row's (oracle sum8_tree; Markstein quotients unless some lane of the wave flags
// an argument below -65, then IEEE division everywhere -- equal results wherever the Markstein quotient is
// exact).  Called by lanes 0-15 of one wave; lanes 0-7 get pp (lane q's prior), value and reward.
struct OneHeads {
  float pp, value, reward;
};
template <bool SUP33>
__device__ __forceinline__ OneHeads one_heads(const MzhOneSmem& sm, int l16, bool recurrent) {
  const int q = l16 & 7;
  const bool rh = l16 >= 8;
  const bool live = SUP33 && (!rh || recurrent);  // this group's head feeds a result (mzh_heads_row: h < nh)
  const float* lv = rh ? sm.lrwd : sm.lval;
  const float lraw = sm.lpol[q];
  const float lg = q < MZH_A ? lraw : -__builtin_inff();
  float e[5], m = -__builtin_inff();
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = q + 8 * i;
    e[i] = (live && k < 33) ? lv[k] : -__builtin_inff();
    m = __builtin_fmaxf(e[i], m);
  }
  const float mp = mzh_max8_nonan(lg);
  m = mzh_max8_nonan(m);
  const float xp = lg - mp;
  const float epx = mzh_expf_np(xp);
  const float ep = q < MZH_A ? epx : 0.0f;
  float xmin = q < MZH_A ? xp : 0.0f;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const float xv = e[i] - m;
    const float ex = mzh_expf_np(xv);
    e[i] = (q + 8 * i < 33) ? ex : 0.0f;
    if (live && q + 8 * i < 33) xmin = __builtin_fminf(xv, xmin);
  }
  float a = e[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) a = a + e[i];
  if (q == 0) a = a + e[4];
  const float sp = mzh_sum8(ep);
  const float sh = mzh_sum8(a);
  const bool slow = xmin < -65.0f;
  auto mdiv = [](float x, float b, float y) {
    const float qq = x * y;
    const float rr = __builtin_fmaf(-qq, b, x);
    return __builtin_fmaf(rr, y, qq);
  };
  float pp = mdiv(ep, sp, 1.0f / sp), pk[5];
  const float y = 1.0f / sh;
#pragma unroll
  for (int i = 0; i < 5; ++i) pk[i] = mdiv(e[i], sh, y);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    pp = ep / sp;
#pragma unroll
    for (int i = 0; i < 5; ++i) pk[i] = e[i] / sh;
  }
  OneHeads out;
  out.pp = q < MZH_A ? pp : 0.0f;
  if (SUP33) {
    float x = 0.0f;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = q + 8 * i;
      if (k < 33) {
        const float prod = pk[i] * (float)(k - 16);
        x = i == 0 ? prod : x + prod;
      }
    }
    x = mzh_sum8(x);
    const float tv = mzh_signed_parabolic(x);
    out.value = tv;
    // the reward head's result, from lane q + 8 (row_ror:8)
    const float tr = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(tv), 0x128, 0xF, 0xF, true));
    out.reward = recurrent ? tr : 0.0f;
  } else {  // support 1 (TD_return = False): the raw head outputs
    out.value = sm.lval[0];
    out.reward = recurrent ? sm.lrwd[0] : 0.0f;
  }
  return out;
}

// normalize_h_state (networks.py:191-196) of the 64 units held one per lane of a full wave: min / max over
// the wave (exact, order-free: DPP within each 16-lane row, then the gfx950 row swaps across rows -- no LDS
// crossbar round trips), IEEE division as the oracle's normalize_h.  The raw units are NaN- and -0-free (an FMA
// chain from +0 plus a bias), so v_min / v_max are the oracle's min / max.
__device__ __forceinline__ float one_rowswap_min(float v, bool b32) {
  const auto r = b32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false)
                     : __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return mzh_vmin(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float one_rowswap_max(float v, bool b32) {
  const auto r = b32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false)
                     : __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return mzh_vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float one_normalize64(float h) {
  float mn = mzh_min8_nonan(h), mx = mzh_max8_nonan(h), a, b;
  asm volatile("s_nop 1\n\tv_min_f32_dpp %0, %1, %1 row_mirror row_mask:0xf bank_mask:0xf" : "=v"(a) : "v"(mn));
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 row_mirror row_mask:0xf bank_mask:0xf" : "=v"(b) : "v"(mx));
  mn = one_rowswap_min(one_rowswap_min(a, false), true);
  mx = one_rowswap_max(one_rowswap_max(b, false), true);
  const float d = (mx - mn) + 9.999999939225290290778502821922302246094e-09f;
  return (h - mn) / d;
}

// LDS past the output layers: tree blocks | UCB table, RN(1/k) | path snapshots + chain values | path |
// (LATL) the latents
struct OneLayout {
  size_t table, pc, pcv, path, lat, total;
};
__host__ __device__ inline OneLayout one_layout(int S, bool latl) {
  OneLayout L;
  L.table = kTreeOff + (size_t)(S + 1) * sizeof(MzhBlock);  // tree blocks (block 0 = the root: unused)
  L.pc = L.table + sizeof(double) * 2 * (size_t)(S + 3);
  L.pcv = L.pc + sizeof(MzhPathEnt) * (size_t)(S + 1);
  L.path = L.pcv + sizeof(double) * (size_t)(S + 1);
  L.lat = (L.path + sizeof(uint16_t) * (size_t)(S + 1) + 15) & ~(size_t)15;
  L.total = L.lat + (latl ? sizeof(float) * MZH_H * (size_t)(S + 1) : 0);
  return L;
}
}  // namespace

size_t mzh_one_smem_bytes(int S, bool latl) { return (one_layout(S, latl).total + 15) & ~(size_t)15; }

// The root's 8-lane group (wave 0, lanes 0-7; lane c = child slot c) over the LDS tree.  The same operations,
// in the same order, as MzhTree (mzh_tree.h) -- node.py:53-123's arithmetic in fp64 with the shared helpers --
// only the storage differs: every block in LDS, the path a flat array.
struct MzhOneTree {
  const MzhSearchParams& p;
  MzhRootBlk& rb;
  MzhBlock* tb;
  uint16_t* path;
  MzhPathEnt* pc;  // [S + 1] the picked child's (W, R, N) at each depth, snapshot by the selection
  double* pcv;     // [S + 1] the value the backup adds at each depth
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
    if (c == pick) {
      path[0] = (uint16_t)pick;
      pc[0] = MzhPathEnt{rb.W[c], rb.R[c], Nr};
    }
    int depth = 1, e = 0;
    const int cs = c < MZH_A ? c : MZH_A - 1;
    MZH_LSTAMP_DECL
    while ((nx >> 16) >= 0) {
      e = nx >> 16;
      const int Np = nx & 0xFFFF;
      const MzhBlock& b = tb[e];
      int nxc = *reinterpret_cast<const int*>(&b.sl[cs].nx);
      const float Rc = b.sl[cs].R, Pc = b.sl[cs].P;
      const double Wc = b.W[cs];
      if (c >= MZH_A) nxc = (int)0xFFFF0000;
      const int Nc = nxc & 0xFFFF;
#ifdef MZH_STAMPS
      asm volatile("" ::"v"(nxc), "v"(Rc), "v"(Pc), "v"(Wc));
#endif
      MZH_LSTAMP(0);
      {
        const float u = mzh_ucb(Nc, Wc, Rc, (double)Pc, p.np1, table[Np], disc, has, mmin, den, dinv, inv, EXACT);
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
      nx = mzh_group_take(nxc, c == pick);
      if (c == pick) {
        path[depth] = (uint16_t)(e * 8 + pick);
        pc[depth] = MzhPathEnt{Wc, Rc, Nc};
      }
      depth++;
#ifdef MZH_STAMPS
      asm volatile("" ::"v"(nx));
#endif
      MZH_LSTAMP(3);
      MZH_LSTAMP_COUNT();
    }
    MZH_LSTAMP_FLUSH(20);
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
    MZH_LSTAMP_DECL
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
    // the fp64 value chain leaf -> root on every lane (node.py:53-70: W += value, then value = rwd + gamma *
    // value), from the rewards the selection snapshot; lane j % 8 keeps the value added at depth j
    MZH_LSTAMP(0);
    double v = (double)val;
    for (int j = depth - 1; j >= 0; --j) {
      const double rw = j == depth - 1 ? (double)rew : (double)pc[j].R;
      if (c == (j & 7)) pcv[j] = v;
      v = rw + disc * v;
    }
#ifdef MZH_STAMPS
    asm volatile("" ::"v"(v));
#endif
    MZH_LSTAMP(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // the path nodes' updates, lane c for depths c, c + 8, ...: the snapshot (W, N) + the chain value
    double lmax = -__builtin_inf(), lmin = __builtin_inf();
    for (int j = c; j < depth; j += 8) {
      const int ent = path[j];
      const int e = j == 0 ? 0 : ent >> 3, a = j == 0 ? ent : ent & 7;
      const MzhPathEnt pe = pc[j];
      const double rw = j == depth - 1 ? (double)rew : (double)pe.R;
      const double Wn = pe.W + pcv[j];
      const int Nn = pe.N + 1;
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
#ifdef MZH_STAMPS
    asm volatile("" ::"v"(lmax), "v"(lmin));
#endif
    MZH_LSTAMP(2);
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
#ifdef MZH_STAMPS
    asm volatile("" ::"v"(rs.dinv));
#endif
    MZH_LSTAMP(3);
    MZH_LSTAMP_COUNT();
    MZH_LSTAMP_FLUSH(14);
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

// LATL: the latents in LDS (when the launcher finds room; otherwise in the engine's HBM workspace)
template <bool SUP33, bool MMIN, bool LATL>
__global__ __launch_bounds__(512, 2) void mzh_search_one_kernel(MzhNet net, MzhOneNet on, MzhSearchParams p) {
  extern __shared__ __align__(128) unsigned char smem_raw[];
  MzhOneSmem& sm = *reinterpret_cast<MzhOneSmem*>(smem_raw);
  float4* l2 = reinterpret_cast<float4*>(smem_raw + kSmBytes);
  const float* l2f = reinterpret_cast<const float*>(smem_raw + kSmBytes);
  MzhBlock* tb = reinterpret_cast<MzhBlock*>(smem_raw + kTreeOff);
  const int S = p.S;
  const OneLayout lay = one_layout(S, LATL);
  double* table = reinterpret_cast<double*>(smem_raw + lay.table);
  double* inv = table + (S + 3);  // inv[k] = RN(1/k), k <= S + 2
  MzhPathEnt* pc = reinterpret_cast<MzhPathEnt*>(smem_raw + lay.pc);
  double* pcv = reinterpret_cast<double*>(smem_raw + lay.pcv);
  uint16_t* path = reinterpret_cast<uint16_t*>(smem_raw + lay.path);
  float* latl = reinterpret_cast<float*>(smem_raw + lay.lat);  // LATL: [S + 1][64]

  const int t = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform (scalar branches)
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
  for (int i = t; i < (int)(sizeof(MzhOneSmem) / 4); i += kThreads) reinterpret_cast<float*>(&sm)[i] = 0.0f;
  for (int i = t; i < S + 3; i += kThreads) {
    table[i] = i < S + 2 ? p.table[i] : 0.0;
    inv[i] = 1.0 / (double)i;  // IEEE division: correctly rounded
  }
  const double disc = p.discount;
  const bool noised = p.noise != nullptr;
  __syncthreads();

  for (int r = blockIdx.x; r < p.B; r += gridDim.x) {
    // this root's latents [E][64] in the engine's workspace: lane j stores and re-reads element j
    const __amdgpu_buffer_rsrc_t lres = mzh_rsrc(p.htree + (size_t)r * p.E * MZH_H);
    const int tr = one_fresh(t), lane = tr & 63, n = tr & 255, c = lane & 7;
    const bool grp = wave == 0 && lane < 8;  // the root's 8-lane group (tree phases)
    MzhOneTree tree{p, sm.root, tb, path, pc, pcv, table, inv, lane, disc, noised};
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
      sm.hidDT[one_t256(n)] = one_relu(acc + on.rep0b[n]);
    }
    __syncthreads();
    if (wave == 0) {  // representation_net.2 + normalize_h_state
      const float h = one_chain256<64>(l2 + MZH_ONE_D2, sm.hidDT, lane, lane) + on.rep2b[lane];
      const float hn = one_normalize64(h);
      sm.xhT[one_t64(lane)] = hn;
      if (LATL)
        latl[lane] = hn;  // node 0's latent
      else
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hn), lres, 4 * lane, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i)
      *reinterpret_cast<floatx4*>(&l2[MZH_ONE_D2 + tr + 512 * i]) =
          mzh_ld4(l2res, 16 * tr, 16 * (MZH_ONE_D2 + 512 * i));
    if (!A) {  // prediction hidden layers
      float xr[4], ap = 0.0f, av = 0.0f;
      one_rows<4>(xr, sm.xhT, lane);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (v == 0)
          one_fma16<true>(ap, xr[v], w1);
        else
          one_fma16(ap, xr[v], w1 + 16 * v);
        one_fma16(av, xr[v], w2 + 16 * v);
      }
      const float hv = one_relu(av + b1b);
      sm.hidPT[one_t256(n)] = one_relu(ap + b1a);
      sm.hidVT[one_t256(n)] = hv;
      sm.hidVQ[one_q(n)] = hv;
    }
    __syncthreads();
    if (wave == 0 && lane >= 32) {  // value_net.2 bins 0-31
      const float acc = one_chain256<64>(l2 + MZH_ONE_A2, sm.hidVT, lane, lane);
      sm.lval[lane - 32] = acc + l2f[MZH_ONE_B2 * 4 + 64 + lane];
    } else if (wave == 1 && lane < 16) {  // policy_net.2 (rows 8-15 repeat 0-7: a DPP row needs all 16 lanes)
      const float acc = one_chain256<8>(l2 + MZH_ONE_P2, sm.hidPT, lane & 7, lane);
      if (lane < MZH_A) sm.lpol[lane] = acc + l2f[MZH_ONE_B2 * 4 + 128 + lane];
    } else if (SUP33 && wave == 2 && lane >= 4 && lane < 8) {  // value bin 32: four chains over k = g mod 4
      const int g = lane & 3;
      float acc = one_chain_bin32(sm.hidVQ + 68 * g, l2f + MZH_ONE_C32 * 4 + 64 * lane);
      acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0xB1, 0xF, 0xF, true));  // p0+p1 | p2+p3
      acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x4E, 0xF, 0xF, true));
      if (lane == 4) sm.lval[32] = acc + l2f[MZH_ONE_B2 * 4 + 137];
    }
    __syncthreads();
    OneHeads ho{0.0f, 0.0f, 0.0f};
    if (wave == 0 && lane < 16) ho = one_heads<SUP33>(sm, lane, false);
    if (grp) {
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
      MzhRootReg rs;
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
      if (c == 0) sm.rsv = rs;
    }
    int lsum = 0;  // p.lockstep_levels: this root's selection levels below the root, summed
    if (wave == 0 && S > 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      const int e = sm.rsv.leafE, a = sm.rsv.leafA;
      lsum += sm.rsv.depth - 1;
      // the leaf's parent latent (mcts.py:89-92), stored by this lane
      sm.xlT[one_t64(lane)] =
          LATL ? latl[e * MZH_H + lane]
               : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lres, 4 * lane, 4 * MZH_H * e, 0));
      if (lane == 0) sm.act = a;
    }
    __syncthreads();
    MZH_STAMP_DECL
    for (int s = 0; s < S; ++s) {
      const int ts = one_fresh(t), ls = ts & 63, ns = ts & 255;
      // ---------------- expand via the network (mcts.py:88-106, networks.py:96-150) ----------------
      if (A) {  // dynamic_net.0: 64 latent steps, the one-hot column, bias, ReLU
        const int a = sm.act;
        float acc = one_chain64(w1, sm.xlT, ls);
        const float wa = a == 0 ? woh[0] : a == 1 ? woh[1] : a == 2 ? woh[2] : a == 3 ? woh[3] : a == 4 ? woh[4] : woh[5];
        acc = acc + wa;
        sm.hidDT[one_t256(ns)] = one_relu(acc + b1a);
      }
      MZH_STAMP(1);
      __syncthreads();
      MZH_STAMP(2);
      if (wave == 0) {  // dynamic_net.2 (K = 256), then normalize_h_state
        const float hr = one_chain256<64>(l2 + MZH_ONE_D2, sm.hidDT, ls, ls) + l2f[MZH_ONE_B2 * 4 + ls];
        sm.hrawT[one_t64(ls)] = hr;
        const float hn = one_normalize64(hr);
        sm.xhT[one_t64(ls)] = hn;
        if (LATL)
          latl[(s + 1) * MZH_H + ls] = hn;  // the new node's latent (expanded node s + 1)
        else
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hn), lres, 4 * ls, 4 * MZH_H * (s + 1), 0);
      }
      MZH_STAMP(3);
      __syncthreads();
      MZH_STAMP(4);
      if (A) {  // rwd_net.0 on the un-normalised latent
        const float hr = one_relu(one_chain64(w2, sm.hrawT, ls) + b1b);
        sm.hidRT[one_t256(ns)] = hr;
        sm.hidRQ[one_q(ns)] = hr;
      } else {  // policy_net.0 / value_net.0 on the normalised latent
        float xr[4], ap = 0.0f, av = 0.0f;
        one_rows<4>(xr, sm.xhT, ls);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          if (v == 0)
            one_fma16<true>(ap, xr[v], w1);
          else
            one_fma16(ap, xr[v], w1 + 16 * v);
          one_fma16(av, xr[v], w2 + 16 * v);
        }
        const float hv = one_relu(av + b1b);
        sm.hidPT[one_t256(ns)] = one_relu(ap + b1a);
        sm.hidVT[one_t256(ns)] = hv;
        sm.hidVQ[one_q(ns)] = hv;
      }
      MZH_STAMP(5);
      __syncthreads();
      MZH_STAMP(6);
      if (wave == 0) {  // rwd_net.2 bins 0-31 (lanes 0-31) | value_net.2 bins 0-31 (lanes 32-63)
        const float acc = one_chain256<64>(l2 + MZH_ONE_A2, ls < 32 ? sm.hidRT : sm.hidVT, ls, ls);
        const float y = acc + l2f[MZH_ONE_B2 * 4 + 64 + ls];
        if (ls < 32)
          sm.lrwd[ls] = y;
        else
          sm.lval[ls - 32] = y;
      } else if (wave == 1 && ls < 16) {  // policy_net.2 (rows 8-15 repeat 0-7: a DPP row needs all 16 lanes)
        const float acc = one_chain256<8>(l2 + MZH_ONE_P2, sm.hidPT, ls & 7, ls);
        if (ls < MZH_A) sm.lpol[ls] = acc + l2f[MZH_ONE_B2 * 4 + 128 + ls];
      } else if (SUP33 && wave == 2 && ls < 8) {  // bin 32 of both heads: lane 4h + g runs chain g of head h
        const int g = ls & 3;
        float acc = one_chain_bin32((ls < 4 ? sm.hidRQ : sm.hidVQ) + 68 * g, l2f + MZH_ONE_C32 * 4 + 64 * ls);
        acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0xB1, 0xF, 0xF, true));
        acc = acc + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc), 0x4E, 0xF, 0xF, true));
        if (ls == 0) sm.lrwd[32] = acc + l2f[MZH_ONE_B2 * 4 + 136];
        if (ls == 4) sm.lval[32] = acc + l2f[MZH_ONE_B2 * 4 + 137];
      }
      MZH_STAMP(7);
      __syncthreads();
      MZH_STAMP(8);
      // ---------------- heads, backup (node.py:53-70), the next selection ----------------
      OneHeads hs{0.0f, 0.0f, 0.0f};
      if (wave == 0 && ls < 16) hs = one_heads<SUP33>(sm, ls, true);
      if (grp) {
        const OneHeads ho = hs;
        MzhRootReg rs = sm.rsv;
        MZH_STAMP(9);
        tree.backup(ls & 7, s, rs, ho.value, ho.reward, ho.pp);
        MZH_STAMP(10);
        if (s + 1 < S) {
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
          __builtin_amdgcn_wave_barrier();
          tree.template select<MMIN>(ls & 7, rs);
        }
        if ((ls & 7) == 0) sm.rsv = rs;
        MZH_STAMP(11);
      }
      if (wave == 0 && s + 1 < S) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
        const int e = sm.rsv.leafE, a = sm.rsv.leafA;
        lsum += sm.rsv.depth - 1;
        sm.xlT[one_t64(ls)] =
            LATL ? latl[e * MZH_H + ls]
                 : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lres, 4 * ls, 4 * MZH_H * e, 0));
        if (ls == 0) sm.act = a;
      }
      MZH_STAMP(12);
      __syncthreads();
      MZH_STAMP(13);
    }
    // ---------------- results (mcts.py:111-126, 154-176) ----------------
    if (wave == 0 && lane == 0) {
      const MzhRootReg rs = sm.rsv;
      tree.results(r, rs);
      if (p.lockstep_levels) p.lockstep_levels[r] = lsum;
    }
    __syncthreads();  // the next root reuses the LDS tree and activations
  }
}

template <bool SUP33, bool MMIN, bool LATL>
static hipError_t launch_one_t(const MzhNet& net, const MzhOneNet& on, const MzhSearchParams& p, int grid,
                               hipStream_t stream) {
  const size_t smem = mzh_one_smem_bytes(p.S, LATL);
  const void* fn = reinterpret_cast<const void*>(&mzh_search_one_kernel<SUP33, MMIN, LATL>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((mzh_search_one_kernel<SUP33, MMIN, LATL>), dim3(grid), dim3(kThreads), smem, stream, net, on, p);
  return hipGetLastError();
}
template <bool SUP33, bool MMIN>
static hipError_t launch_one_l(const MzhSearchPlan& pl, const MzhNet& net, const MzhOneNet& on, const MzhSearchParams& p,
                               hipStream_t stream) {
  return pl.ohl ? launch_one_t<SUP33, MMIN, true>(net, on, p, pl.grid, stream)
                : launch_one_t<SUP33, MMIN, false>(net, on, p, pl.grid, stream);
}

// the instantiation the plan names (grid = min(B, 256): one round of workgroups, each persistent over its roots;
// pl.ohl: the latents in LDS)
hipError_t mzh_launch_one(const MzhSearchPlan& pl, const MzhNet& net, const MzhOneNet& on, const MzhSearchParams& p,
                          hipStream_t stream) {
  if (pl.sup33) return pl.mmin ? launch_one_l<true, true>(pl, net, on, p, stream) : launch_one_l<true, false>(pl, net, on, p, stream);
  return pl.mmin ? launch_one_l<false, true>(pl, net, on, p, stream) : launch_one_l<false, false>(pl, net, on, p, stream);
}

#ifdef MZH_STAMPS
// diagnostic build only: this file's phase stamps [8 waves][MZH_NSTAMP], read and cleared
extern "C" int mzh_diag_stamps_one(unsigned long long* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(mzh_stamp_acc), sizeof(mzh_stamp_acc)) != hipSuccess) return -2;
  static unsigned long long zero[8][MZH_NSTAMP] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(mzh_stamp_acc), zero, sizeof(zero)) != hipSuccess) return -2;
  return 0;
}
#endif
