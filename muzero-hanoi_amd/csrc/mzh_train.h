// mzh_train.h -- parameter blocks of the fused training update (mzh_train.hip), filled by the C
// ABI (mzh_api.hip: mzh_train_update).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/mzh.h"

// kernel-1 view of the network (names follow networks.py:39-67): every weight both as torch stores
// it ([out][in]) and transposed ([in][out], suffix T), so that each GEMV direction reads coalesced
struct MztNet {
  const float *rep1, *rep1T, *rep1b, *rep2, *rep2T, *rep2b;
  const float *dyn1, *dyn1T, *dyn1b, *dyn2, *dyn2T, *dyn2b;
  const float *rwd1, *rwd1T, *rwd1b, *rwd2, *rwd2T, *rwd2b;
  const float *pol1, *pol1T, *pol1b, *pol2, *pol2T, *pol2b;
  const float *val1, *val1T, *val1b, *val2, *val2T, *val2b;
};

// per-layer inputs X and output gradients GY, rows m = b * U + t (step layers) or b (representation)
struct MztScratch {
  float *x0;    // [B][32]     observation, zero-padded
  float *repa;  // [B][256]    representation hidden activation
  float *h;     // [BU][64]    h_t (normalised), input of policy / value / dynamics layer 1
  float *ap, *av, *ad, *ar;  // [BU][256] hidden activations
  float *hp;    // [BU][64]    h'_{t+1} (before normalisation), input of reward layer 1
  float *g_rep; // [B][256]    representation hidden pre-activation gradient
  float *g_h0p; // [B][64]     representation output gradient
  float *g_p, *g_v, *g_d, *g_r;  // [BU][256] hidden pre-activation gradients
  float *g_lp;  // [BU][16]    policy logit gradient (zero-padded)
  float *g_lv, *g_lr;  // [BU][48 | 16] value / reward logit gradients (zero-padded)
  float *g_hp;  // [BU][64]    dynamics output gradient
};

struct MztRowParams {
  int B, U, in_dim;
  const float *obs, *rwds, *pi, *returns, *w;
  const int64_t* actions;
  float* row_loss;  // [B][3]
  float* new_prio;  // [B] or null
  MztNet n;
  MztScratch s;
};

struct MztGradLayer {
  const float* X;
  int ldx;
  const float* GY;
  int ldg;
  int M, out, in;
  int onehot_from;  // columns >= onehot_from are the one-hot action (dynamics layer 1), else -1
  int tile0, nkb;   // first tile of this layer in the grid, 16-column blocks of `in`
  float *W, *b, *mW, *vW, *mb, *vb;
  float* WT;        // transposed copy [in][ldwt] to refresh
  int ldwt;         // out rounded up to a multiple of 4 (16-byte rows)
};

struct MztGradParams {
  MztGradLayer L[10];
  const int64_t* actions;
  float step_size, bc2_sqrt, beta1, beta2, eps;
};

size_t mzt_rows_smem_bytes(int rows, int U);
hipError_t mzt_launch_rows(int rows, int support, const MztRowParams& p, hipStream_t stream);
hipError_t mzt_launch_grad_adam(const MztGradParams& P, int n_tiles, hipStream_t stream);
hipError_t mzt_launch_transpose(const float* W, float* WT, int out, int in, int ldwt, hipStream_t stream);

// prioritised replay on the device (mzh_replay.hip): the draw + gather and the priority write-back
#define MZR_MAX_BATCH 4096  // batch_s per draw (the sampled indices sit in LDS)
hipError_t mzr_launch_sample(const mzh_replay_args& a, hipStream_t stream);
hipError_t mzr_launch_set_priorities(float* prio, long long size, const int64_t* idx, const float* val, int m,
                                     int32_t* status, hipStream_t stream);
