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
  const float* rp_pi;
  const float* rp_reward;
  const float* rp_value;
  unsigned char* tree;  // [B][E] MzhBlock
  float* htree;         // [B][E][64]
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
};

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
    if (r < nvalid) p.h[(size_t)(row0 + r) * MZH_H + k] = sm.x[r * MZH_LD64 + k];
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

size_t mzh_search_smem_bytes(int R, int S);
hipError_t mzh_launch_search(int R, bool replay, const MzhNet& net, const MzhSearchParams& p, hipStream_t stream);
hipError_t mzh_launch_infer(int R, bool recurrent, const MzhNet& net, const MzhInferParams& p, hipStream_t stream);
