// mzh_env_kernels.h -- launchers of the environment kernels (mzh_env.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

hipError_t mzh_launch_env_step(int n, int goal_peg, int max_steps, int B, uint8_t* state, const int32_t* action,
                               uint8_t* moved, float* obs, int8_t* reward, uint8_t* done, uint8_t* illegal,
                               int32_t* step_ctr, uint8_t* active, int32_t* err_count, hipStream_t s);
hipError_t mzh_launch_legal_mask(int n, int B, const uint8_t* state, uint8_t* mask, hipStream_t s);
hipError_t mzh_launch_encode_obs(int n, int B, const uint8_t* state, float* obs, hipStream_t s);
hipError_t mzh_launch_hanoi_solver(int n, int goal_peg, int B, const uint8_t* state, int32_t* moves, hipStream_t s);
