// mzh_search.hip -- fused batched MuZero search + batched MLP inference kernels (gfx950).
//
// One workgroup (256 threads = 4 waves) owns R = 16*MT roots and runs ALL of their simulations:
//   select  : 8 lanes per root, one lane per child; fp64 Q / UCB exactly as MCTS/node.py:72-123,
//             6-way argmax + tie detection by shuffles/ballot inside the 8-lane group
//   expand  : recurrent_inference for the R pending leaves as fp32 MFMA GEMMs (mzh_device.h)
//   backup  : one lane per root walks the LDS path leaf -> root (MCTS/node.py:53-70)
// Roots are independent (one owner per tree): no atomics, no inter-workgroup traffic, one launch
// per search.  Trees live in HBM as flat blocks (mzh_tree.h: one 128-B line per expanded node
// holding its 6 children's N/X/R/P/W); the per-sim path, per-root min-max, root stats, UCB table and
// the MLP activations live in LDS.  Weights stream from L2 (shared by every workgroup of an XCD).
#include "mzh_device.h"
#include "mzh_internal.h"
#include "mzh_tree.h"

// One workgroup per CU (all 512 registers per lane): the next simulation's first weight chunks stay
// in flight across the tree phase.  Overlapping one root group's tree phase with another's MLP was
// measured slower in both forms tried: two co-resident 16-root workgroups per CU
// (<= 256 registers, no cross-phase prefetch) and a 512-thread workgroup whose waves 0-3 run the MLP
// of one 16-root half while waves 4-7 run the other half's tree work (the co-resident tree work
// took twice as long as alone) -- a v_mfma_f32_16x16x4_f32 stream holds its SIMD's vector issue, so a
// partner wave's tree work stalls beside it (tools/micro/overlap_probe.hip).  The 32-root tile on 8
// waves with both waves of a SIMD in the same phase lost 9% too.
//
// Per simulation: the MLP (all four waves split every layer's output tiles, activations in LDS),
// one barrier, then each root's own 8-lane group runs -- with no further workgroup barrier -- the
// heads of its row, the backup of this simulation and the selection of the next one, then one
// barrier.  Tree-phase mapping: root r = wave * (R / 4) + lane / 8, child slot c = lane % 8, so the
// tree work of R = 16 roots is spread over all four waves as well.
template <int R>
constexpr int search_dc() { return R == 32 ? 16 : 32; }  // LDS-cached path depths

// MMIN: the launch has caller-given MinMaxStats bounds (p.minmax_in), which could make max - min
// subnormal: the selection then checks for that (MzhTree::select)
// C8: the two-workgroups-per-CU form (mzh_search_occ2_kernel): 16-root tile, <= 256 registers, the MLP
// on 8-fragment weight chunks (mzh_mlp_recurrent_c8), DC = 16 cached path depths, no one-hot in LDS
template <int R, int DC, bool C8, bool REPLAY, bool OHL, bool SUP33, bool MMIN>
__device__ __forceinline__ void mzh_search_body(const MzhNet& net, const MzhSearchParams& p) {
  static_assert(!C8 || (R == 16 && !OHL), "the 8-fragment MLP is the 16-root tile's");
  constexpr int NF = C8 ? 8 : 16;  // fragments per weight buffer
  using Smem = SearchSmem<R, DC>;
  // tree-phase waves: all four (R / 4 roots each), or for C8 two full waves of 8 roots -- waves 0-1 of one
  // workgroup of a CU's pair, waves 2-3 of the other (workgroups b and b + 256 share a CU when 512 of them
  // fill 256 CUs two deep), so each SIMD runs one 8-root tree wave per simulation as in the 32-root tile
  // instead of two half-empty ones (the pairing is a placement guess: correctness does not depend on it)
  constexpr int TRW = C8 ? 2 : 4;
  constexpr int RPW = R / TRW;  // roots per tree wave
  constexpr int N2 = SUP33 ? 2 : 1;  // rwd2 / val2 MFMA tiles (bin 32 of a 33-bin head: vector chains)
  extern __shared__ __align__(16) unsigned char smem_raw[];
  MlpSmem<R>& sm = *reinterpret_cast<MlpSmem<R>*>(smem_raw);
  Smem& st = *reinterpret_cast<Smem*>(smem_raw + sizeof(MlpSmem<R>));
  double* table = reinterpret_cast<double*>(smem_raw + sizeof(MlpSmem<R>) + sizeof(Smem));
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
  // this lane's root (tree phases) and child slot
  const int tw = C8 ? wave - ((blockIdx.x >> 8) & 1) * 2 : wave;  // tree-wave index (wave-uniform)
  const int tr = tw * RPW + (lane >> 3), tc = lane & 7;
  const bool tgroup = (unsigned)tw < (unsigned)TRW && (lane >> 3) < RPW;  // wave-uniform per 8-lane group

  if (OHL)
    for (int i = tid; i < MZH_A * MZH_F; i += MZH_THREADS) ohl[i] = net.dyn0_onehot[i];
  if (SUP33 && !REPLAY) mzh_w32_fill<R>(sm, net, tid);
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
    st.tie[r] = (p.tie_idx && r < nvalid) ? p.tie_idx[root0 + r] : 0;
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
      sm.x[r * MZH_LD64 + mzh_kpos(k)] = (r < nvalid && k < p.in_dim) ? p.obs[(size_t)(root0 + r) * p.in_dim + k] : 0.0f;
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
  floatx4 fa[NF], fb[NF];
  float ba[4], bb[4];
  if (!REPLAY) {
    if constexpr (C8)
      mzh_mlp_fetch12_c8(sm, net, wave, lane, fa, ba, fb, bb);
    else
      mzh_mlp_fetch12<R>(sm, net, wave, lane, fa, ba, fb, bb);
  }
  __syncthreads();

  MzhTree<R, DC, REPLAY, MlpSmem<R>> tree{p, st, sm, path, table, inv, root0, PL, lane, disc, noised};

  // within a root's 8-lane group: LDS and tree stores of one step are visible to the next step
  auto group_sync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
  };

  // the root's state lives in its group's registers from here to the results
  MzhRootReg rs;
  const bool town = tgroup && tr < nvalid;
  if (town) rs.load(st, tr);

  // p.lockstep_levels: the workgroup's deepest selection below the root per simulation (every wave's
  // maximum through LDS, read by thread 0 after the simulation's closing barrier).  Selection k writes
  // slot k & 1: without an MLP (replay) the other waves may finish selection k + 1 before thread 0 has
  // read selection k's maxima, but selection k + 2 -- the next writer of that slot -- starts only after
  // the barrier that thread 0 reaches once it has read them
  const bool lcount = p.lockstep_levels != nullptr;
  int lsum = 0;
  auto wave_level = [&](int k) {
    int m = town ? rs.depth - 1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
    if (lane == 0) st.lvl[k & 1][wave] = m;
  };
  auto group_level = [&](int k) {
    int m = st.lvl[k & 1][0];
#pragma unroll
    for (int w = 1; w < MZH_WAVES; ++w) m = max(m, st.lvl[k & 1][w]);
    lsum += m;
  };
  MZH_STAMP_DECL
  if (town) tree.template select<MMIN>(tr, tc, 0, rs);
  if (lcount) wave_level(0);
  __syncthreads();
  if (lcount && tid == 0 && S > 0) group_level(0);
  for (int s = 0; s < S; ++s) {
    // ---------------- expand via the network (mcts.py:88-106) ----------------
    if (!REPLAY) {
      MZH_STAMP(19);
      if constexpr (C8) {
        // the previous simulation's last chunks loaded this one's A1 / A2 into the swapped buffers
        if (s > 0) mzh_c8_swap(fa, ba, fb, bb);
        mzh_mlp_recurrent_c8<N2>(sm, net, wave, lane, fa, ba, fb, bb, net.dyn0_onehot);
      } else {
        mzh_mlp_recurrent_body<R, true, N2, false>(sm, net, wave, lane, fa, ba, fb, bb, OHL ? ohl : net.dyn0_onehot);
      }
      MZH_STAMP(20);
    }
    if (town) {
      const int r = tr, c = tc;
      // this row's heads (networks.py:83,109,152-189) or its recorded network outputs, in registers
      MzhHeadOut ho;
      if (!REPLAY) {
        ho = mzh_heads_row<R, SUP33 ? 33 : 0, false, !SUP33>(sm, net, r, c, net.support, true);
      } else {
        const float* rec = p.rp_sim + ((size_t)s * p.B + root0 + r) * 8;  // 6 priors, reward, value
        ho.pp = c < MZH_A ? rec[c] : 0.0f;
        ho.reward = rec[6];
        ho.value = rec[7];
      }
      MZH_STAMP(21);
      tree.backup(r, c, s, rs, ho.value, ho.reward, ho.pp);
      MZH_STAMP(22);
      if (s + 1 < S) {
        group_sync();
        tree.template select<MMIN>(r, c, s + 1, rs);
        MZH_STAMP(30);
      }
    }
    if (lcount && s + 1 < S) wave_level(s + 1);
    __syncthreads();
    if (lcount && tid == 0 && s + 1 < S) group_level(s + 1);
    MZH_STAMP(23);
  }
  if (lcount && tid == 0) p.lockstep_levels[blockIdx.x] = lsum;

  // ---------------- results (mcts.py:111-126, 154-176) ----------------
  if (town && tc == 0) rs.store(st, tr);
  __syncthreads();
  if (tid < R * 8) {
    const int r = tid >> 3, c = tid & 7;
    if (r < nvalid && c == 0) tree.results(r);
  }
}

template <int R, bool REPLAY, bool OHL, bool SUP33, bool MMIN>
__global__ __launch_bounds__(MZH_THREADS, 1) void mzh_search_kernel(MzhNet net, MzhSearchParams p) {
  mzh_search_body<R, search_dc<R>(), false, REPLAY, OHL, SUP33, MMIN>(net, p);
}

// Two 16-root workgroups per CU (<= 256 registers, <= 80 KB LDS each): while one runs its MLP's MFMA
// chains the other's tree phase (dependent block loads, fp64 chains) fills the SIMDs' stalls
template <bool SUP33, bool MMIN>
__global__ __launch_bounds__(MZH_THREADS, 2) void mzh_search_occ2_kernel(MzhNet net, MzhSearchParams p) {
  mzh_search_body<16, 16, true, false, false, SUP33, MMIN>(net, p);
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
    sm.x[r * MZH_LD64 + mzh_kpos(k)] = (r < nvalid && k < p.in_dim) ? p.x[(size_t)(row0 + r) * p.in_dim + k] : 0.0f;
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
    sm.x[r * MZH_LD64 + mzh_kpos(k)] = r < nvalid ? p.x[(size_t)(row0 + r) * MZH_H + k] : 0.0f;
  }
  if (tid < R) sm.act[tid] = tid < nvalid ? p.action[row0 + tid] : 0;
  __syncthreads();
  mzh_mlp_recurrent<R>(sm, net, wave, lane);
  mzh_store_outputs<R>(sm, p, row0, nvalid, net.support, true);
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <int R, int DC = search_dc<R>()>
static size_t search_smem_bytes(int S, bool ohl) {
  size_t b = sizeof(MlpSmem<R>) + sizeof(SearchSmem<R, DC>);
  b += sizeof(double) * 2 * (size_t)(S + 3);
  b += sizeof(uint16_t) * (size_t)((R * (S + 1) + 7) & ~7);
  if (ohl) b += sizeof(float) * MZH_A * MZH_F;
  return (b + 15) & ~(size_t)15;
}

template <int R, bool REPLAY, bool OHL, bool SUP33, bool MMIN>
static hipError_t launch_search_m(const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const size_t smem = search_smem_bytes<R>(p.S, OHL);
  const void* fn = reinterpret_cast<const void*>(&mzh_search_kernel<R, REPLAY, OHL, SUP33, MMIN>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int grid = (p.B + R - 1) / R;
  hipLaunchKernelGGL((mzh_search_kernel<R, REPLAY, OHL, SUP33, MMIN>), dim3(grid), dim3(MZH_THREADS), smem, stream, net,
                     p);
  return hipGetLastError();
}
template <int R, bool REPLAY, bool OHL, bool SUP33>
static hipError_t launch_search_s(const MzhSearchPlan& pl, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  // caller-given bounds: the instantiation that checks for a subnormal max - min (MzhTree::select)
  if (pl.mmin) return launch_search_m<R, REPLAY, OHL, SUP33, true>(net, p, stream);
  return launch_search_m<R, REPLAY, OHL, SUP33, false>(net, p, stream);
}
template <int R, bool REPLAY, bool OHL>
static hipError_t launch_search_t(const MzhSearchPlan& pl, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  // the replay kernel never runs the network: one instantiation (SUP33 = true) serves both supports
  if (REPLAY || pl.sup33) return launch_search_s<R, REPLAY, OHL, true>(pl, net, p, stream);
  return launch_search_s<R, REPLAY, OHL, false>(pl, net, p, stream);
}

// the LDS a search launch needs at tile R (ohl: with the dynamics one-hot columns in LDS; occ2: the
// two-workgroups-per-CU kernel, 16 cached path depths)
size_t mzh_search_smem_bytes(int R, int S, bool ohl, bool occ2) {
  if (occ2) return search_smem_bytes<16, 16>(S, false);
  return R == 32 ? search_smem_bytes<32>(S, ohl) : search_smem_bytes<16>(S, ohl);
}

template <bool SUP33, bool MMIN>
static hipError_t launch_search_occ2(const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  const size_t smem = search_smem_bytes<16, 16>(p.S, false);
  const void* fn = reinterpret_cast<const void*>(&mzh_search_occ2_kernel<SUP33, MMIN>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  const int grid = (p.B + 15) / 16;
  hipLaunchKernelGGL((mzh_search_occ2_kernel<SUP33, MMIN>), dim3(grid), dim3(MZH_THREADS), smem, stream, net, p);
  return hipGetLastError();
}

// the instantiation the plan names (mzh_api.hip make_plan decides every template argument)
hipError_t mzh_launch_search(const MzhSearchPlan& pl, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream) {
  if (pl.occ2) {
    if (pl.sup33) return pl.mmin ? launch_search_occ2<true, true>(net, p, stream) : launch_search_occ2<true, false>(net, p, stream);
    return pl.mmin ? launch_search_occ2<false, true>(net, p, stream) : launch_search_occ2<false, false>(net, p, stream);
  }
  if (pl.R == 32) {
    if (pl.replay) return launch_search_t<32, true, false>(pl, net, p, stream);
    if (pl.ohl) return launch_search_t<32, false, true>(pl, net, p, stream);
    return launch_search_t<32, false, false>(pl, net, p, stream);
  }
  if (pl.replay) return launch_search_t<16, true, false>(pl, net, p, stream);
  if (pl.ohl) return launch_search_t<16, false, true>(pl, net, p, stream);
  return launch_search_t<16, false, false>(pl, net, p, stream);
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
