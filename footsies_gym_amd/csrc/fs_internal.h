// Internal interface between the host C-ABI (fs_api.cpp) and the HIP kernels
// (fs_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/footsies.h"

namespace fsk {

// BattleAI's input plans (AI:192-312): the queue of a plan holds plan_len inputs, so a queue
// index is always below its plan's length (host validation and the kernels' code tables).
enum { MP_NEUTRAL, MP_FAR1, MP_FAR2, MP_MID1, MP_MID2, MP_FALLBACK1, MP_FALLBACK2 };
enum { AP_NONE, AP_ONE_HIT, AP_TWO_HIT, AP_IMMEDIATE_SPECIAL, AP_DELAY_SPECIAL };
constexpr uint32_t move_plan_len(uint32_t plan) {  // AI:192-253
  return plan == MP_FAR1 ? 90u : plan == MP_FAR2 ? 56u : plan == MP_MID1 ? 70u : plan == MP_MID2 ? 33u
       : plan == MP_FALLBACK1 ? 60u : plan == MP_FALLBACK2 ? 63u : 30u;
}
constexpr uint32_t attack_plan_len(uint32_t plan) {  // AI:255-312
  return plan == AP_ONE_HIT ? 19u : plan == AP_TWO_HIT ? 23u : plan == AP_IMMEDIATE_SPECIAL ? 61u
       : plan == AP_DELAY_SPECIAL ? 121u : 30u;
}

// Per-arena state in HBM, struct-of-arrays (one element per arena, 8/16-byte
// vectors so one wave64 load/store moves 512 B / 1 KiB contiguous).
struct DevState {
  float2* pos;     // x of P1, P2 (Fighter.position.x)
  uint2* hist;     // per fighter: bit j = backward on input[j], bit 16 + j = forward (facing-relative)
  uint4* fpk;      // packed fighter words: (P1 lo, P1 hi, P2 lo, P2 hi), layout in fs_kernels.hip
  int2* aw;        // (frameCount, arena header word)
  double* cum;     // FootsiesEnv._cummulative_episode_reward
  uint4* rng;      // the game's UnityEngine.Random Xorshift128 state (every mode)
  uint2* bot;      // P2's BattleAI: (bot word, previous FightState distance bits), layout in fs_kernels.hip
  uint2* bot1;     // P1's BattleAI (FS_P1_BOT), same layout
  float2* posy;    // y of P1, P2 (Fighter.position.y): 0 unless a state load set it (general geometry)
};

// The kernels' P2 variants.  FS_P2_EXTERNAL / FS_P2_BOT / FS_P2_NOOP run handles whose actors are
// fixed and uniform (P1 the agent; P2 remote, the bot, or idle); kActors runs per-arena actors: a
// P1 bot (FS_P1_BOT) and / or P2 switched between remote and bot (fs_set_p2_mode).
constexpr int kActors = 3;

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
  // fs_step_n_packed (include/footsies.h fs_packed_traj): lane records of 16 B, with `reward`
  // above as the trajectory's reward; the per-field pointers are then unused
  uint4* pk_lanes;
  uint4* pk_final;
};

// the in-kernel actor of fs_step_n_policy (fs_policy.h): fp32 weights in torch layouts
struct PolicyParams {
  const float *w1, *b1, *w2, *b2, *w3, *b3;  // [64][8] [64] [64][64] [64] [8][64] [8]
  uint8_t* actions;  // [n][N] or null
  float* logp;       // [n][N] or null
  uint64_t seed;
};

struct StepParams {
  DevState st;
  DevOutputs out;
  PolicyParams pol;
  const uint8_t* p1;   // [n][N] or null (hashed)
  const uint8_t* p2;   // [n][N] or null
  const uint8_t* active;  // [N] or null: single-tick launches skip arenas whose byte is 0
  uint64_t action_seed;
  uint64_t t0;         // global step index of the first tick (hash counter)
  uint64_t arena_base; // global index of arena 0 (fs_config.arena_base): hash / sampling keys
  int n_envs;
  int n_steps;
  int out_stride_steps;  // 1: outputs are [n][N] trajectories; 0: overwrite one [N] set
  int dense_reward;
  int autoreset_mode;
  int p1_bot;     // kActors: P1 is the bot (FS_P1_BOT)
  int p2_resets;  // kActors: P2's bot is Reset at Intro (the handle was created with FS_P2_BOT)
  int p2_noop;    // kActors: a non-bot P2 presses nothing (FS_P2_NOOP handle)
  int prio;       // fused launches: time-sliced wave priority (set by the launcher, prio_slice)
  int geom;       // some arena has position.y != 0 or a flipped facing: the general-geometry tick
  int prefetch;   // two-lane fused row launches: each tick's request prepared at the end of the tick before
  uint2* rec;     // one-tick launches (fs_step_rec): each arena's FS_RECORD_BYTES record, or null
  // host actions of a one-tick launch over at most kInlineArenas arenas, carried in the kernel
  // arguments instead of a staging copy (inl_n != 0): byte a of inl[player] is arena a's input
  int inl_n;
  uint32_t inl[2][8];
};
constexpr int kInlineArenas = 32;  // sizeof(StepParams::inl[0])

struct ResetParams {
  DevState st;
  DevOutputs out;
  const uint64_t* seeds;  // [N] or null
  const uint8_t* mask;    // [N] or null
  int n_envs;
  int flags;
  int init;  // 1: fresh arenas (`new Fighter()`), seeds from base_seed
  uint64_t base_seed;
  uint64_t arena_base;
  int p1_bot, p2_mode;  // the handle's actors (fs_config p1_mode / p2_mode)
};

// FootsiesEnv's delayed-frame queue (FE:126-131, 493-504, 532-535) for frame_delay = d > 0:
// per arena a ring of d packed observation records, slot = global step index mod d
// (all arenas step together).  Applied after a step kernel to the rows it wrote, or
// after a reset to refill the rings of fresh arenas (output frame == -1).
struct DelayParams {
  DevOutputs out;
  uint4* ring;          // [d][N] records of 2 x uint4 (layout in fs_delay.hip)
  int n_envs;
  int delay;            // d
  int n_steps;          // rows to process (1 for fs_step / fs_reset)
  int out_stride_steps;
  uint8_t* head;        // [N] per arena: the ring slot its next step reads and overwrites
  const uint8_t* active;  // fs_step_masked: only these arenas stepped (nullptr = all)
  int refill_only;      // 1: after fs_reset / fs_create (no queue shift)
  int same_step;        // FS_AUTORESET_SAME_STEP: a terminal row's final_* take the delayed record
};

// launchers (fs_kernels.hip, fs_delay.hip); return hipError_t of the launch
// variant: FS_P2_EXTERNAL / FS_P2_BOT / FS_P2_NOOP or kActors (see above)
hipError_t launch_step(const StepParams& p, int float_mode, int variant, hipStream_t s);
const char* step_kernel_name(bool policy, bool hashed, int n_steps, int n_envs, int float_mode, int variant,
                             bool geom, bool packed, int autoreset_mode);
hipError_t launch_reset(const ResetParams& p, int float_mode, hipStream_t s);
hipError_t launch_set_p2(const DevState& st, int bot, const uint8_t* mask, int n, hipStream_t s);
hipError_t launch_hash_actions(int n_envs, int n_steps, uint64_t seed, uint64_t t0, uint64_t arena_base, uint8_t* p1,
                               uint8_t* p2, hipStream_t s);
hipError_t launch_get_state(const DevState& st, fs_arena_state* dst, fs_env_state* env_dst, int n, hipStream_t s);
hipError_t launch_set_state(const DevState& st, const fs_arena_state* src, int n, hipStream_t s);
hipError_t launch_delay(const DelayParams& p, hipStream_t s);
hipError_t launch_pack_records(const DevOutputs& o, void* dst, int n, hipStream_t s);
// fs_learn.hip: the C5 learner's minibatch gradient (fs_ppo_grad)
size_t ppo_workspace_bytes();
hipError_t launch_ppo_grad(const float* rows, int64_t n, const float* const actor[6], const float* const critic[6],
                           float clip, float vf_coef, float ent_coef, float* grad, float* loss, void* workspace,
                           hipStream_t s, bool split, const int64_t* runs = nullptr, int run_shift = 0,
                           int64_t n_rows = 0);
hipError_t launch_ppo_eval(const float* x, int64_t n_values, const uint8_t* actions, int64_t n_logp,
                           const float* const actor[6], const float* const critic[6], float* values, float* logp,
                           void* workspace, hipStream_t s, bool split);
hipError_t launch_ppo_gae(const double* rew, const uint8_t* done, const float* val, int T, int64_t N, float gamma,
                          float gamma_lam, float* adv, float* ret, hipStream_t s);
hipError_t launch_ppo_features(const uint8_t* guard, const uint8_t* move, const float* move_frame,
                               const float* position, int64_t n, float* out, hipStream_t s);
hipError_t launch_ppo_pack(const float* x, const uint8_t* act, const float* old, const float* adv, const float* ret,
                           const float* stats, int64_t n, float* rows, hipStream_t s);

}  // namespace fsk
