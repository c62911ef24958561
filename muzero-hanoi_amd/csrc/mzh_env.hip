// mzh_env.hip -- Tower-of-Hanoi environment kernels (env/hanoi.py, utils.py:9-25,
// env/hanoi_utils.py:4-26), one lane per env, integer-only, bit-exact with the reference.
//
// A state is N bytes (peg of disc d, disc 0 smallest), the reference's tuple layout.  The legal
// test _move_allowed (hanoi.py:123-139: from-peg non-empty and (to-peg empty or min(to) >
// min(from))) is computed as top[f] < top[t] with top[p] = smallest disc on peg p (N if empty).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mzh_env_kernels.h"

#define MZH_MAXN 32

__constant__ int8_t kMoveFrom[6] = {0, 0, 1, 1, 2, 2};  // permutations(range(3), 2),
__constant__ int8_t kMoveTo[6] = {1, 2, 0, 2, 0, 1};    // env/hanoi.py:39-41

__device__ __forceinline__ void load_state(const uint8_t* src, int n, uint8_t* st, int top[3]) {
  top[0] = top[1] = top[2] = n;
  for (int d = n - 1; d >= 0; --d) {
    st[d] = src[d];
    top[st[d]] = d;
  }
}

__global__ void mzh_env_step_kernel(int n, int goal_peg, int max_steps, int B, uint8_t* state,
                                    const int32_t* action, uint8_t* moved, float* obs, int8_t* reward,
                                    uint8_t* done, uint8_t* illegal, int32_t* step_ctr, uint8_t* active,
                                    int32_t* err_count) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  uint8_t st[MZH_MAXN];
  int top[3];
  load_state(state + (size_t)b * n, n, st, top);
  const int a = action[b];
  int8_t code;
  uint8_t dn = 0, ill = 0;
  if (!active[b] || a < 0 || a >= 6) {
    // assert self.reset_check (hanoi.py:49) / moves[action] IndexError: env left untouched
    code = -2;
    if (err_count) atomicAdd(err_count, 1);
  } else {
    const int f = kMoveFrom[a], t = kMoveTo[a];
    ill = !(top[f] < top[t]);
    int ctr = step_ctr[b] + 1;  // hanoi.py:61
    if (!ill) {
      const int disc = top[f];  // smallest disc on the from-peg (hanoi.py:148-150)
      st[disc] = (uint8_t)t;
      bool goal = true;
      for (int d = 0; d < n; ++d) goal = goal && (st[d] == goal_peg);
      if (!goal) {
        code = 0;
        state[(size_t)b * n + disc] = (uint8_t)t;  // c_state = moved_state
      } else {
        code = 1;  // rwd 100, done, reset_check False, counter 0; c_state NOT advanced (hanoi.py:65-69)
        dn = 1;
        active[b] = 0;
        ctr = 0;
      }
    } else {
      code = -1;  // rwd -100/1000, state unchanged (hanoi.py:70-74)
    }
    if (ctr == max_steps) {  // hanoi.py:77-80
      dn = 1;
      active[b] = 0;
      ctr = 0;
    }
    step_ctr[b] = ctr;
  }
  reward[b] = code;
  done[b] = dn;
  illegal[b] = ill;
  if (moved)
    for (int d = 0; d < n; ++d) moved[(size_t)b * n + d] = st[d];
  if (obs) {
    float* o = obs + (size_t)b * 3 * n;
    for (int d = 0; d < n; ++d) {
      o[3 * d + 0] = st[d] == 0 ? 1.0f : 0.0f;
      o[3 * d + 1] = st[d] == 1 ? 1.0f : 0.0f;
      o[3 * d + 2] = st[d] == 2 ? 1.0f : 0.0f;
    }
  }
}

__global__ void mzh_legal_mask_kernel(int n, int B, const uint8_t* state, uint8_t* mask) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  uint8_t st[MZH_MAXN];
  int top[3];
  load_state(state + (size_t)b * n, n, st, top);
  uint8_t m = 0;
  for (int a = 0; a < 6; ++a) m |= (uint8_t)((top[kMoveFrom[a]] < top[kMoveTo[a]]) << a);
  mask[b] = m;
}

__global__ void mzh_encode_obs_kernel(int n, int B, const uint8_t* state, float* obs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // one lane per (env, disc)
  if (i >= B * n) return;
  const uint8_t s = state[i];
  float* o = obs + (size_t)i * 3;
  o[0] = s == 0 ? 1.0f : 0.0f;
  o[1] = s == 1 ? 1.0f : 0.0f;
  o[2] = s == 2 ? 1.0f : 0.0f;
}

__global__ void mzh_hanoi_solver_kernel(int n, int goal_peg, int B, const uint8_t* state, int32_t* moves) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint8_t* st = state + (size_t)b * n;
  int32_t m = 0;
  int target = goal_peg;
  for (int i = n - 1; i >= 0; --i) {  // env/hanoi_utils.py:18-24
    if (st[i] != target) {
      m += 1 << i;
      target = 3 - target - st[i];
    }
  }
  moves[b] = m;
}

static inline int nblocks(int work, int tpb) { return (work + tpb - 1) / tpb; }

hipError_t mzh_launch_env_step(int n, int goal_peg, int max_steps, int B, uint8_t* state, const int32_t* action,
                               uint8_t* moved, float* obs, int8_t* reward, uint8_t* done, uint8_t* illegal,
                               int32_t* step_ctr, uint8_t* active, int32_t* err_count, hipStream_t s) {
  hipLaunchKernelGGL(mzh_env_step_kernel, dim3(nblocks(B, 256)), dim3(256), 0, s, n, goal_peg, max_steps, B, state,
                     action, moved, obs, reward, done, illegal, step_ctr, active, err_count);
  return hipGetLastError();
}

hipError_t mzh_launch_legal_mask(int n, int B, const uint8_t* state, uint8_t* mask, hipStream_t s) {
  hipLaunchKernelGGL(mzh_legal_mask_kernel, dim3(nblocks(B, 256)), dim3(256), 0, s, n, B, state, mask);
  return hipGetLastError();
}

hipError_t mzh_launch_encode_obs(int n, int B, const uint8_t* state, float* obs, hipStream_t s) {
  hipLaunchKernelGGL(mzh_encode_obs_kernel, dim3(nblocks(B * n, 256)), dim3(256), 0, s, n, B, state, obs);
  return hipGetLastError();
}

hipError_t mzh_launch_hanoi_solver(int n, int goal_peg, int B, const uint8_t* state, int32_t* moves, hipStream_t s) {
  hipLaunchKernelGGL(mzh_hanoi_solver_kernel, dim3(nblocks(B, 256)), dim3(256), 0, s, n, goal_peg, B, state, moves);
  return hipGetLastError();
}
