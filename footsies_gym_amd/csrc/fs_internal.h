// Internal interface between the host C-ABI (fs_api.cpp) and the HIP kernels
// (fs_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/footsies.h"

namespace fsk {

// Per-arena state in HBM, struct-of-arrays (one element per arena, 8/16-byte
// vectors so one wave64 load/store moves 512 B / 1 KiB contiguous).
struct DevState {
  float2* pos;     // x of P1, P2 (Fighter.position.x)
  uint2* hist;     // Left/Right bits of input[0..15] per fighter, input[0] in bits 0-1
  uint4* fpk;      // packed fighter words: (P1 lo, P1 hi, P2 lo, P2 hi), layout in fs_kernels.hip
  int2* aw;        // (frameCount, arena header word)
  double* cum;     // FootsiesEnv._cummulative_episode_reward
  uint4* rng;      // bot: UnityEngine.Random Xorshift128 state
  uint2* bot;      // bot: (queue word, previous FightState distance bits)
};

struct DevOutputs {
  uint8_t* guard;
  uint8_t* move;
  float* move_frame;
  float* position;
  double* reward;
  uint8_t* terminated;
  uint8_t* truncated;
  int32_t* frame;
  uint8_t* action;
  uint8_t* hitstun;
  uint8_t* final_guard;
  uint8_t* final_move;
  float* final_move_frame;
  float* final_position;
  int32_t* final_frame;
  uint8_t* final_action;
  uint8_t* final_hitstun;
};

struct StepParams {
  DevState st;
  DevOutputs out;
  const uint8_t* p1;   // [n][N] or null (hashed)
  const uint8_t* p2;   // [n][N] or null
  uint64_t action_seed;
  uint64_t t0;         // global step index of the first tick (hash counter)
  int n_envs;
  int n_steps;
  int out_stride_steps;  // 1: outputs are [n][N] trajectories; 0: overwrite one [N] set
  int dense_reward;
  int autoreset_mode;
};

struct ResetParams {
  DevState st;
  DevOutputs out;
  const uint64_t* seeds;  // [N] or null
  const uint8_t* mask;    // [N] or null
  int n_envs;
  int flags;
  int init;  // 1: fresh arenas (`new Fighter()`), seeds from base_seed
  uint64_t base_seed;
};

// launchers (fs_kernels.hip); return hipError_t of the launch
hipError_t launch_step(const StepParams& p, int float_mode, int p2_mode, hipStream_t s);
hipError_t launch_reset(const ResetParams& p, int float_mode, int p2_mode, hipStream_t s);
hipError_t launch_hash_actions(int n_envs, int n_steps, uint64_t seed, uint64_t t0, uint8_t* p1, uint8_t* p2,
                               hipStream_t s);
hipError_t launch_get_state(const DevState& st, fs_arena_state* dst, fs_env_state* env_dst, int n, int p2_mode,
                            hipStream_t s);
hipError_t launch_set_state(const DevState& st, const fs_arena_state* src, int n, int p2_mode, hipStream_t s);

}  // namespace fsk
