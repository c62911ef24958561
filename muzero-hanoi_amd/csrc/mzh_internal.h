// mzh_internal.h -- parameter blocks shared by the launchers (mzh_search.hip) and the C ABI
// implementation (mzh_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mzh_device.h"

struct MzhSearchParams {
  int B, S, E;          // roots, simulations, tree blocks per root (engine max_sims + 1)
  int in_dim, kin;      // observation width 3N and its zero-padded width (16 * rep0.kb)
  int deterministic, np1;
  double discount, eps, temperature;
  const float* obs;
  const double* noise;
  const int32_t* tie_idx;
  const double* action_u;
  const double* minmax_in;
  const float* rp_root_pi;
  const float* rp_sim;  // [S][B][8] replay records (6 priors, reward, value)
  unsigned char* tree;  // [B][E] MzhBlock
  float* htree;         // [B][E][64]
  uint16_t* pathx;      // [B][E] selection-path slots beyond the LDS-cached depths (wave kernel)
  const double* table;  // [S+2] UCB table (log((n+19653)/19652)+1.25)*sqrt(n)
  int32_t* visits;
  double* root_q;
  double* minmax_out;
  int32_t* extra_ties;
  int32_t* action;
  double* pi;
  int32_t* latent;
  int32_t* latent_len;
  int32_t* sel_steps;
  const double* pow_table;  // [S + 1] np.power(n, 1/T) for a non-integer exponent (nullable)
  int32_t* lockstep_levels;  // [groups] sum over simulations of each lockstep group's deepest selection (nullable)
};

// visits ** e as generate_play_policy computes it (np.power(int64 visits, e), mcts.py:168-174), for
// x = n visits and e = max(1, min(5, 1/T)): an integer exponent is an exact product (n^5 < 2^53);
// a non-integer one is taken from pow_table[n], the caller's np.power(arange(S + 1), e) (NumPy's
// vectorised pow -- SVML on AVX-512 hosts -- differs from any other pow in the last bit for some
// n), or from the device pow when no table is given
__device__ __forceinline__ double mzh_pow(double x, int n, double e, const double* pow_table) {
  if (e == __builtin_rint(e)) {
    double r = x;
    for (int i = 1; i < (int)e; ++i) r = r * x;
    return r;
  }
  return pow_table ? pow_table[n] : pow(x, e);
}

struct MzhInferParams {
  int B, in_dim, kin;
  const float* x;         // obs [B][in_dim] (initial) or h [B][64] (recurrent)
  const int32_t* action;  // [B] (recurrent)
  float* h;
  float* reward;
  float* pi;
  float* value;
  float* policy_logits;
  float* value_logits;
  float* reward_logits;
};

template <int R>
__device__ __forceinline__ void mzh_store_outputs(MlpSmem<R>& sm, const MzhInferParams& p, int row0, int nvalid,
                                                  int support, bool recurrent) {
  const int tid = threadIdx.x;
  for (int i = tid; i < R * MZH_H; i += MZH_THREADS) {
    const int r = i >> 6, k = i & 63;
    if (r < nvalid) p.h[(size_t)(row0 + r) * MZH_H + k] = sm.x[r * MZH_LD64 + mzh_kpos(k)];
  }
  for (int i = tid; i < R * 8; i += MZH_THREADS) {
    const int r = i >> 3, c = i & 7;
    if (r < nvalid && c < MZH_A) {
      if (p.pi) p.pi[(size_t)(row0 + r) * MZH_A + c] = sm.pi[r * 8 + c];
      if (p.policy_logits) p.policy_logits[(size_t)(row0 + r) * MZH_A + c] = sm.lpol[r * MZH_LDPOL + c];
    }
  }
  for (int i = tid; i < R * support; i += MZH_THREADS) {
    const int r = i / support, k = i - r * support;
    if (r < nvalid) {
      if (p.value_logits) p.value_logits[(size_t)(row0 + r) * support + k] = sm.lval[r * MZH_LDSUP + k];
      if (recurrent && p.reward_logits) p.reward_logits[(size_t)(row0 + r) * support + k] = sm.lrwd[r * MZH_LDSUP + k];
    }
  }
  if (tid < nvalid) {
    if (p.value) p.value[row0 + tid] = sm.value[tid];
    if (p.reward) p.reward[row0 + tid] = sm.reward[tid];
  }
}

// ------------------------------------------------------------------------------------------
// Wave-kernel network layout (mzh_wave.hip).  Each MLP (layer1 -> ReLU -> layer2) is one stream
// of MFMA A-fragments with the WEIGHTS as the A operand and the activations (one root per
// column) as the B operand, so a hidden tile's C registers feed the next layer's B operand
// directly (no LDS round trip).  Per hidden tile ht (16 units) the stream holds KB1 layer-1
// fragments then NO layer-2 fragments, each [64 lanes] float4:
//   layer1 frag (ht, kb)[lane][t] = W1[u(ht, lane&15)][16kb + 4t + (lane>>4)]
//   layer2 frag (ht, ot)[lane][t] = W2[pi(ot, lane&15)][16ht + 4t + (lane>>4)]
// with u(ht, r) = 16ht + 4(r&3) + (r>>2): C row 4g+i of hidden tile ht is unit 16ht + 4i + g, which
// is exactly the unit lane group g must supply at k-step i of layer 2 -- every dot product stays
// a k-ordered fp32 FMA chain from 0 (the numerics contract of mzh_device.h).  One zero ht block
// pads the stream end (unconditional prefetch).  b1/b2 are the biases in C-register order.
// ------------------------------------------------------------------------------------------
struct MzhWMlp {
  const float4* s;  // [17][KB1 + NO][64]
  const float* b1;  // [256]: b1[16ht + 4g + i] = bias1[16ht + 4i + g]
  const float* b2;  // [16 NO]: b2[16ot + 4g + i] = bias2[pi(ot, 4g + i)] (0 on padding rows)
  // 33-bin heads: bins 0..31 in the NO = 2 tiles, bin 32 as four vector-FMA chains (lane group g: hidden
  // units 16ht + 4t + g, t = 0..3): w32[4ht + g] = those units' weights, b32 its bias (MzhNet::rwd32)
  const float4* w32;
  float b32;
  int kb1, no;
  int soff, b1off, b2off, w32off;  // byte offsets of s, b1, b2, w32 in the packed blob (MzhWNet::wbase)
};
struct MzhWNet {
  MzhWMlp rep, dyn, rwd, pol, val;
  const float* wbase;  // the packed weight blob: one buffer resource serves every chain's loads
  const float* oh;  // [6][256]: oh[a][16ht + 4g + i] = dynamic_net.0.weight[u(ht, 4g + i)][64 + a]
  int support, in_dim;
};

// ------------------------------------------------------------------------------------------
// Latency-path network layout (mzh_one.hip: one root per workgroup, weights stationary on the CU).
// The hidden layers' rows live in registers for the whole launch: thread t < 256 holds unit t of
// dynamic_net.0 (64 latent + 6 one-hot columns) and rwd_net.0, thread 256 + t unit t of policy_net.0 and
// value_net.0.  The K = 256 output layers live in LDS, copied verbatim from `l2` (k-major: one
// ds_read_b128 gives a lane the 4 k-steps of its output row, 1 KiB contiguous per wave).
//   l1 [66 k4][256 units] float4: k4 0-15 dynamic_net.0 latent columns, 16-31 rwd_net.0, 32-47 policy_net.0,
//      48-63 value_net.0, 64-65 dynamic_net.0 one-hot columns 64..69 (+ 2 zero)
//   b1 [256] float4 {dynamic_net.0, rwd_net.0, policy_net.0, value_net.0} bias of the unit
//   rep0 [in_dim][256] representation_net.0 (k-major), rep2 [64 k4][64] float4 representation_net.2
//   l2: the LDS image, MZH_ONE_* offsets in float4 units
// ------------------------------------------------------------------------------------------
#define MZH_ONE_D2 0                        // dynamic_net.2 [64 k4][64 lanes]
#define MZH_ONE_A2 (64 * 64)                // rwd_net.2 bins 0-31 (lanes 0-31) | value_net.2 bins 0-31 (lanes 32-63)
#define MZH_ONE_P2 (2 * 64 * 64)            // policy_net.2 [64 k4][8 lanes] (6 rows + 2 zero)
#define MZH_ONE_C32 (MZH_ONE_P2 + 64 * 8)   // bin 32 chains [8 lanes][64 i] floats: lane g < 4 the reward head's
                                            // chain g (k = g + 4i), lane 4 + g the value head's (128 float4)
#define MZH_ONE_B2 (MZH_ONE_C32 + 128)      // biases (floats): [0,64) dynamic_net.2, [64,128) the A2 rows,
                                            // [128,136) policy_net.2, 136 / 137 bin 32 of reward / value
#define MZH_ONE_L2F4 (MZH_ONE_B2 + 36)      // float4s of the LDS image
struct MzhOneNet {
  const float4* l1;
  const float4* b1;
  const float* rep0;
  const float* rep0b;
  const float4* rep2;
  const float* rep2b;
  const float4* l2;
};

// Every template argument of one search launch, decided once on the host (mzh_api.hip make_plan) and
// used both to launch and to report the launched instantiation (mzh_search_plan_query)
struct MzhSearchPlan {
  int wave;    // 1: mzh_wave_kernel<nt, replay, sup33>; 0: mzh_search_kernel<R, replay, ohl, sup33, mmin>
  int nt;      // wave kernel: 16-root column tiles per wave
  int R;       // cooperative kernel: roots per workgroup
  int replay;  // tree-only instantiation (recorded network outputs)
  int ohl;     // cooperative: the dynamics one-hot columns in LDS; one: the latents in LDS
  int sup33;   // 33-bin value / reward support (cooperative replay: always 1, one instantiation)
  int mmin;    // cooperative / one: caller-given MinMaxStats bounds (subnormal max - min check)
  int occ2;    // cooperative: mzh_search_occ2_kernel<sup33, mmin> (16-root tile, two workgroups per CU)
  int one;     // latency path: mzh_search_one_kernel<sup33, mmin, ohl> (one root per workgroup)
  int grid;    // one: workgroups (each loops over roots b, b + grid, ...)
};

size_t mzh_one_smem_bytes(int S, bool latl);
hipError_t mzh_launch_one(const MzhSearchPlan& pl, const MzhNet& net, const MzhOneNet& on, const MzhSearchParams& p,
                          hipStream_t stream);
size_t mzh_wave_smem_bytes(int S, int nt);
hipError_t mzh_launch_wave_search(const MzhSearchPlan& pl, const MzhWNet& net, const MzhSearchParams& p, hipStream_t stream);
size_t mzh_search_smem_bytes(int R, int S, bool ohl, bool occ2 = false);
hipError_t mzh_launch_search(const MzhSearchPlan& pl, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream);
hipError_t mzh_launch_infer(int R, bool recurrent, const MzhNet& net, const MzhInferParams& p, hipStream_t stream);
