/*
 * footsies.h -- C-ABI of libfootsies.so, the MI355X-native vectorized FOOTSIES
 * simulator (HIP kernels for gfx950).
 *
 * The reference has no native FFI for this path: its boundary is a Python
 * gymnasium.Env (FootsiesEnv) talking over TCP to a Unity process.  Every entry
 * point below replaces one piece of that stack for N independent arenas at once;
 * the piece is cited next to it (paths relative to the reference root,
 * FE = footsies-gym/footsies_gym/envs/footsies.py, BC = Assets/Script/BattleCore.cs).
 *
 * Conventions
 *   - plain C types only; no exceptions cross the ABI; every call returns 0 on
 *     success or a negative FS_E_* code, with a message via fs_last_error();
 *   - one handle = one device + one HIP stream; calls on a handle must be
 *     serialised by the caller, different handles may run on different threads;
 *   - the library allocates and owns its device buffers; caller buffers are
 *     borrowed for the duration of the call only (unless bound with
 *     fs_bind_outputs, see below);
 *   - fs_step / fs_step_n / fs_reset are asynchronous on the handle's stream;
 *     fs_sync() or the caller's own stream sync orders host reads.
 */
#ifndef FOOTSIES_H
#define FOOTSIES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FS_ABI_VERSION 7

/* error codes */
#define FS_OK 0
#define FS_E_INVALID (-1)      /* bad argument (FE:100-108 raises ValueError for bad ctor args) */
#define FS_E_DEVICE (-2)       /* HIP runtime failure / no device */
#define FS_E_UNSUPPORTED (-3)  /* configuration not implemented */
#define FS_E_OOM (-4)
#define FS_E_RUNTIME (-5)      /* fs_create found no device and two HIP / HSA runtime images in the process */

/* P2 controller (GameManager.cs:183-190: --p2-bot / remote actor; FE:234-247) */
#define FS_P2_EXTERNAL 0  /* P2 action supplied every step (FE `opponent` callable / remote actor) */
#define FS_P2_BOT 1       /* the in-game scripted BattleAI (BattleAI.cs:10-403) as TrainingBattleAIActor */
#define FS_P2_NOOP 2      /* P2 input always 0 */

/* P1 controller (GameManager.cs:185-200; FE:118, 230-232 `by_example`) */
#define FS_P1_EXTERNAL 0  /* P1 action supplied every step (the agent, TrainingRemoteActor) */
#define FS_P1_BOT 1       /* by_example: the in-game BattleAI plays P1 (--p1-bot --p1-spectator); the
                             agent only observes.  Both bots draw from the game's one UnityEngine.Random,
                             P1 first (TrainingManager.cs:59-77).  The spectator wrapper is not a
                             TrainingBattleAIActor, so P1's BattleAI is never Reset (BC:274-275) */

/* Float evaluation model of the C# arithmetic (parity-unpinned: no Unity binary here) */
#define FS_FLOAT_STRICT32 0  /* every float expression rounded to IEEE binary32 per operation (default) */
#define FS_FLOAT_DOUBLE 1    /* expression temporaries in binary64, rounded to binary32 on store/call */

/* Auto-reset of terminated arenas inside fs_step (the Unity KO->End->Stop->Intro->Fight
 * burst, BC:212-243 / 247-345, which the reference runs without waiting for the agent) */
#define FS_AUTORESET_SAME_STEP 0  /* gymnasium 0.29 SyncVectorEnv: obs = state(-1), final_* = terminal obs */
#define FS_AUTORESET_NEXT_STEP 1  /* gymnasium 1.x: the step after a terminal one runs the burst only */

/* fs_step flags */
#define FS_ACT_HOST 0    /* action pointers are host memory (copied H2D on the handle's stream) */
#define FS_ACT_DEVICE 1  /* action pointers are device memory */

/* fs_reset flags */
#define FS_RESET_HARD 0         /* RESET remote-control command (BC:143-146): Stop->Intro->Fight now */
#define FS_RESET_IF_NEEDED 1    /* FootsiesEnv.reset (FE:482-515): RESET only arenas whose
                                   has_terminated flag is clear; the others just finish the
                                   pending KO->...->Fight burst (if any) and report state(-1) */
#define FS_RESET_SEED_ONLY 2    /* SEED command alone (BC:170-173): Random.InitState on the masked
                                   arenas, nothing else changes and no outputs are written */

#define FS_MAX_FRAME_DELAY 4096

typedef struct fs_config {
  int32_t num_envs;        /* arenas on this handle (>0) */
  int32_t device_id;       /* HIP device ordinal */
  int32_t p2_mode;         /* FS_P2_* */
  int32_t dense_reward;    /* 1: FE._get_dense_reward (FE:388-405, default FE:50); 0: sparse (FE:382-386) */
  int32_t frame_delay;     /* FE:36, 126-131, 493-504, 532-535: observation/info outputs are those of
                              the state frame_delay steps back (d copies of state(-1) after a reset);
                              reward, terminated and fs_get_env_state are the newest state's.
                              0 .. FS_MAX_FRAME_DELAY */
  int32_t float_mode;      /* FS_FLOAT_* */
  int32_t autoreset_mode;  /* FS_AUTORESET_* */
  int32_t p1_mode;         /* FS_P1_* */
  uint64_t base_seed;      /* arena i's game RNG is seeded with (int32)(base_seed + arena_base + i) at
                              creation (Random.InitState, BC:170-173) */
  uint64_t arena_base;     /* global index of arena 0 when the arenas of one run are sharded over
                              several handles / GPUs: the hashed action stream (fs_step_n,
                              fs_hash_actions), the in-kernel actor's sampling stream and the creation
                              seeds are keyed by the global index, so results do not depend on the
                              sharding.  0 for an unsharded handle */
} fs_config;

/*
 * Per-step outputs, struct-of-arrays, row i = arena i.  Pairs are [N][2]
 * (column 0 = P1, column 1 = P2) exactly like FootsiesEnv's observation tuples
 * (FE:360-368) stacked over arenas.
 */
typedef struct fs_outputs {
  uint8_t* guard;        /* [N][2] obs["guard"]                       (FE:361)              */
  uint8_t* move;         /* [N][2] obs["move"] = FOOTSIES_MOVE_ID_TO_INDEX, DEAD/WIN->STAND (FE:362-365, 537-549) */
  float* move_frame;     /* [N][2] obs["move_frame"], 0 for STAND/FORWARD/BACKWARD (FE:339-358) */
  float* position;       /* [N][2] obs["position"]                    (FE:367)              */
  double* reward;        /* [N]    dense or sparse reward, float64 like FE (FE:382-405)     */
  uint8_t* terminated;   /* [N]    p1Vital==0 or p2Vital==0           (FE:555)              */
  uint8_t* truncated;    /* [N]    always 0                           (FE:569-570)          */
  int32_t* frame;        /* [N]    info["frame"] = globalFrame        (FE:373)              */
  uint8_t* action;       /* [N][2] info["p1_action"/"p2_action"] as 3-bit ints (Left=1, Right=2, Attack=4; state.py:26-36) */
  uint8_t* hitstun;      /* [N][2] info["p1_hitstun"/"p2_hitstun"]   (FE:376-377)          */
  /* FS_AUTORESET_SAME_STEP only: the terminal observation/info of arenas whose
     terminated flag is set this step (other rows are left untouched) */
  uint8_t* final_guard;      /* [N][2] */
  uint8_t* final_move;       /* [N][2] */
  float* final_move_frame;   /* [N][2] */
  float* final_position;     /* [N][2] */
  int32_t* final_frame;      /* [N]    */
  uint8_t* final_action;     /* [N][2] */
  uint8_t* final_hitstun;    /* [N][2] */
} fs_outputs;

/*
 * Raw EnvironmentState of one arena (Assets/Script/EnvironmentState.cs:10-46,
 * built by BattleCore.GetEnvironmentState, BC:449-468).  Used for state-level
 * parity checks and for a wire-compatible JSON server.
 */
typedef struct fs_env_state {
  int32_t p1Vital, p2Vital, p1Guard, p2Guard;
  int32_t p1Move, p1MoveFrame, p2Move, p2MoveFrame;  /* raw actionIDs (0..510) */
  float p1Position, p2Position;
  int32_t globalFrame;
  int32_t p1MostRecentAction, p2MostRecentAction;
  int32_t p1Hitstun, p2Hitstun;
} fs_env_state;

/*
 * Canonical full state of one arena: everything the simulation carries from one
 * frame to the next (Fighter.cs:73-112, BC:56-70, BattleAI.cs:26-32), in a
 * representation-independent form.  Both the HIP path and the CPU oracle export
 * it, so lockstep tests compare hidden state, not only observations.
 */
typedef struct fs_fighter_state {
  float position_x;
  int32_t action_id;            /* raw actionID */
  int32_t action_frame;
  int32_t hit_count;
  int32_t hitstun;
  int32_t vital;
  int32_t guard;
  int32_t buffer_action_id;     /* -1 = none */
  int32_t reserve_action_id;    /* -1 = none */
  uint32_t input_dir_history;   /* Left/Right bits of input[0..15], 2 bits per frame, input[0] in bits 0-1 */
  int32_t attack_hold;          /* consecutive frames input[0..] had Attack, saturating at 63 */
  uint8_t is_input_backward;
  uint8_t is_reserve_proximity_guard;
  uint8_t has_won;
  uint8_t facing_flipped;       /* 0: the player's own facing (P1 right, P2 left: SetupBattleStart, F:124);
                                   1: the other (Fighter.isFaceRight restored by LoadState, F:744) */
  float position_y;             /* Fighter.position.y (F:742): 0 in every state the game reaches by itself;
                                   a loaded y moves every box (TransformToFightRect F:706-719) and is added
                                   to itself by every push (BC:483-519 pass position.y to
                                   ApplyPositionChange, F:331-350) until the next round start (F:123) */
} fs_fighter_state;

typedef struct fs_arena_state {
  fs_fighter_state f[2];
  int32_t frame_count;          /* BattleCore.frameCount */
  int32_t recording_count;      /* currentRecordingInputIndex, saturating at 18000 */
  uint8_t recording_last[2];    /* recordingPnInput[index-1].input */
  uint8_t actor_input[2];       /* TrainingRemoteActor.input of the remote P1 / P2 actors: the last action
                                   received (stale inputs fed to the Intro tick); 0 where that player has no
                                   remote actor (a bot-created P2, FS_P2_NOOP, FS_P1_BOT) */
  uint8_t reset_pending;        /* FS_AUTORESET_NEXT_STEP: terminal, burst not yet run */
  uint8_t has_terminated;       /* FootsiesEnv.has_terminated (FE:191, 508, 563) */
  uint8_t pad0[2];
  double cumulative_reward;     /* FootsiesEnv._cummulative_episode_reward (FE:187) */
  /* The game's UnityEngine.Random (Xorshift128 state).  One per game, shared by both bots; kept and
     seeded in every mode, so a bot switched in later draws from the seeded stream. */
  uint32_t rng[4];
  /* P2's BattleAI (BattleAI.cs:26-32) */
  int32_t move_plan, move_index;     /* moveQueue as (plan id, dequeued count); plan -1 = empty */
  int32_t attack_plan, attack_index; /* attackQueue likewise */
  float prev_distance;          /* BattleAI.fightStates[5] (== previous call's state) */
  int32_t prev_opponent_action; /* raw actionID of the opponent in that FightState */
  /* actors (ABI 2) */
  uint8_t p2_bot;               /* 1: TrainingManager.actorP2 is the bot (FS_P2_BOT handles always; an
                                   FS_P2_EXTERNAL handle after fs_set_p2_mode) */
  uint8_t bot_ready[2];         /* P1 / P2 BattleAI: fightStates[5] is set, i.e. getNextAIInput has run
                                   since construction or Reset (AI:41-47); 0 = its next call returns 0 */
  uint8_t bot_input[2];         /* TrainingBattleAIActor.input of the P1 / P2 bot (its last answer) */
  uint8_t pad1[3];
  /* P1's BattleAI (FS_P1_BOT), fields as P2's */
  int32_t p1_move_plan, p1_move_index;
  int32_t p1_attack_plan, p1_attack_index;
  float p1_prev_distance;
  int32_t p1_prev_opponent_action;
} fs_arena_state;

typedef struct fs_context* fs_handle;

/* Library / ABI version (FS_ABI_VERSION). */
int fs_abi_version(void);

/* The HIP and HSA runtime images mapped into this process, one "hip:<path>" / "hsa:<path>" line
 * each, written NUL-terminated into buf (truncated to len); returns the larger of the two image
 * counts (1 when the process holds one runtime).  fs_create returns FS_E_RUNTIME, naming both
 * paths, when it finds no device and more than one image of either runtime (ABI 7). */
int fs_runtime_images(char* buf, size_t len);

/* Pinned, device-mapped host memory (hipHostMalloc, zero-filled) and its device address, for
 * callers without a device-memory library of their own -- the torch-free Python surface binds its
 * host outputs there (fs_bind_outputs takes *dev); fs_host_free releases it.  fs_memcpy is a
 * synchronous copy between any two addresses the runtime knows (hipMemcpyDefault).  (ABI 7) */
int fs_host_alloc(int device, size_t bytes, void** host, void** dev);
int fs_host_free(void* host);
int fs_memcpy(void* dst, const void* src, size_t bytes);

/* The HIP runtime version the library is bound to (hipRuntimeGetVersion) and the HIP_VERSION it
 * was compiled against, either pointer optional (ABI 7). */
int fs_runtime_version(int* runtime, int* build);

/* Create N arenas on a device and run the game-start sequence (BattleCore.Start
 * + first Stop->Intro->Fight ticks, BC:105-128, 176-200, 262-291) so they sit at
 * state(-1).  Replaces FootsiesEnv.__init__ + _instantiate_game + _connect_to_game
 * (FE:34-290).  Returns FS_E_INVALID for an out-of-range field. */
int fs_create(const fs_config* cfg, fs_handle* out);

/* Reset arenas (FootsiesEnv.reset, FE:482-515).  seeds: optional host array [N]
 * -> Random.InitState((int32)seed) first (SEED command, BC:170-173; FE:487-488);
 * mask: optional host array [N] of 0/1 selecting arenas (NULL = all); flags:
 * FS_RESET_*.  Writes state(-1) observations of the reset arenas into the
 * outputs (reward 0, terminated 0). */
int fs_reset(fs_handle h, const uint64_t* seeds, const uint8_t* mask, int flags);

/* Switch P2 of the masked arenas (host [N] 0/1, NULL = all) between the remote actor
 * (FS_P2_EXTERNAL) and the in-game bot (FS_P2_BOT): the P2_BOT remote-control command
 * (BC:158-167, TrainingRemoteControl.cs:100-102) that FootsiesEnv.set_opponent sends
 * (FE:458-480).  Only for handles created with FS_P2_EXTERNAL -- the reference needs a
 * custom opponent to accept the command (FE:468-470) -- else FS_E_UNSUPPORTED.  The
 * switch applies from the next tick.  The bot keeps its own state while inactive (queues,
 * FightState, last answer), the remote actor its last received action.  Since such a game
 * was launched without --p2-bot, BattleCore's Intro throws before it could Reset the
 * switched-in bot (BC:276-277, GameManager.cs:187), so that bot is never Reset. */
int fs_set_p2_mode(fs_handle h, int mode, const uint8_t* mask);

/* One Fight tick of every arena (FootsiesEnv.step, FE:518-570 -> BC:201-220,
 * 347-364), with auto-reset of terminated arenas per cfg.autoreset_mode.
 * p1_act: [N] 3-bit inputs (Left=1, Right=2, Attack=4; InputData.cs:8-14); ignored (may be
 * NULL) for FS_P1_BOT.
 * p2_act: [N] for FS_P2_EXTERNAL (read for the arenas whose P2 is the remote actor),
 * ignored (may be NULL) otherwise.
 * flags: FS_ACT_HOST or FS_ACT_DEVICE for where the action arrays live. */
int fs_step(fs_handle h, const uint8_t* p1_act, const uint8_t* p2_act, int flags);

/* fs_step for the arenas whose active[i] != 0 only; the others keep their state
 * and their outputs (which then still hold their previous step's values).  This
 * lets arenas advance at their own pace, as N separate FootsiesEnv instances do
 * under a frame-skipping wrapper (wrappers/frame_skip.py:63-80).  active lives
 * where flags says the actions do.  With frame_delay > 0 each arena's delayed-frame
 * queue advances with that arena's own steps (every FootsiesEnv keeps its own deque). */
int fs_step_masked(fs_handle h, const uint8_t* p1_act, const uint8_t* p2_act, const uint8_t* active, int flags);

/* n Fight ticks in one kernel launch (fused rollout).  Actions: device arrays
 * [n][N], or NULL to draw them on device from the counter-based hash
 * a = splitmix64(action_seed ^ env*0x9E3779B97F4A7C15 ^ (t << 1 | player)) & 7
 * with env = cfg.arena_base + i and t = fs_steps_taken(h) + k.  traj: device arrays laid out [n][N] (pairs
 * [n][N][2]) receiving every tick's outputs; traj == NULL writes each tick
 * into the handle's regular outputs (the last tick remains visible; with
 * frame_delay > 0 the n ticks are then launched one by one, since the delayed
 * queue consumes every tick's row).  Trajectory rows are addressed with 32-bit
 * byte offsets, so a call with n * N above 2^29 - 1 arena-ticks runs as several
 * consecutive launches over row ranges of the same buffers, with identical
 * results. */
int fs_step_n(fs_handle h, int n, const uint8_t* p1_act, const uint8_t* p2_act,
              uint64_t action_seed, const fs_outputs* traj);

/* A packed trajectory for fs_step_n_packed: the values of an fs_outputs trajectory in two
 * stores per tick instead of ten.  Row r = t * N + i (tick t, arena i); k = 0 (P1), 1 (P2):
 *   lanes[r][k]: 16 bytes -- byte 0 guard, 1 move, 2 action (3-bit MostRecentAction), 3 hitstun;
 *                bytes 4-7 move_frame (float), 8-11 position (float); bytes 12-15: for k = 0 the
 *                frame (int32), for k = 1 byte 12 terminated, byte 13 truncated, bytes 14-15 zero.
 *   reward[r]:   float64, as fs_outputs.reward.
 *   final_lanes[r][k] (FS_AUTORESET_SAME_STEP; rows of arenas that did not end are left
 *                untouched): the terminal record in the lanes layout, bytes 12-15 of k = 0 the
 *                final frame, of k = 1 zero.
 * lanes and final_lanes must be 16-byte aligned.  Every field equals the corresponding
 * fs_outputs trajectory field of fs_step_n on the same state and actions. */
#define FS_PACKED_LANE_BYTES 16
typedef struct fs_packed_traj {
  void* lanes;        /* [n][N][2][16 B] */
  double* reward;     /* [n][N] */
  void* final_lanes;  /* [n][N][2][16 B]; required in FS_AUTORESET_SAME_STEP */
} fs_packed_traj;

/* fs_step_n with action rows (p1_act required; p2_act as for fs_step_n) into a packed trajectory.
 * FS_E_UNSUPPORTED with frame_delay > 0. */
int fs_step_n_packed(fs_handle h, int n, const uint8_t* p1_act, const uint8_t* p2_act, const fs_packed_traj* traj);

/* The actor of fs_step_n_policy: an MLP 8 -> 64 -> tanh -> 64 -> tanh -> 8 on
 * P1's observation features [guard/3, move/16, move_frame/55, position/4.6] of
 * P1 then P2 (footsies_gym_amd/rollout.py obs_features), fp32 device weights in
 * torch nn.Linear layouts (weight [out][in]), computed in bf16 with f32
 * accumulation.  The action is drawn from softmax(logits) by inverse CDF with
 * u = uniform(seed, env, t) (fs_policy.h policy_uniform), t = fs_steps_taken + k. */
typedef struct fs_policy {
  const float* w1; /* [64][8] */
  const float* b1; /* [64] */
  const float* w2; /* [64][64] */
  const float* b2; /* [64] */
  const float* w3; /* [8][64] */
  const float* b3; /* [8] */
  uint64_t seed;
  uint8_t* actions_out; /* [n][N] device: P1's sampled actions, or NULL */
  float* logp_out;      /* [n][N] device: their log-probabilities, or NULL */
} fs_policy;

/* fs_step_n with P1 driven by the actor `pol` inside the fused tick loop: the
 * whole policy-in-the-loop rollout in one launch.  p2_act:
 * device [n][N] for FS_P2_EXTERNAL, ignored otherwise.  traj as in fs_step_n.
 * FS_E_UNSUPPORTED with frame_delay > 0. */
int fs_step_n_policy(fs_handle h, int n, const fs_policy* pol, const uint8_t* p2_act, const fs_outputs* traj);

/* The C5 learner (footsies_gym_amd/ppo.py, PPOTrainer(learner="hip")): an MLP
 * 8 -> 64 -> tanh -> 64 -> tanh -> out, fp32 device weights in torch nn.Linear layouts. */
typedef struct fs_mlp {
  const float *w1, *b1, *w2, *b2, *w3, *b3;
} fs_mlp;
#define FS_PPO_ACTOR_PARAMS 5256  /* w1 512, b1 64, w2 4096, b2 64, w3 512, b3 8 */
#define FS_PPO_CRITIC_PARAMS 4801 /* w1 512, b1 64, w2 4096, b2 64, w3 64, b3 1 */
/* Device workspace fs_ppo_grad needs (independent of n). */
size_t fs_ppo_workspace_bytes(void);
/* One minibatch's gradient of PPO's loss, in fp32 on `stream` (a hipStream_t, NULL =
 * the null stream), asynchronously.  rows: device [n][12] f32 = features[8], action,
 * old log-probability, advantage, return.  The loss is ppo.py's:
 *   -mean(min(r A, clamp(r, 1 - clip, 1 + clip) A)) + vf_coef mean((v - R)^2)
 *   - ent_coef mean(H(softmax(actor(x)))),  r = exp(log p(action) - old),
 * actor with 8 outputs (logits), critic with 1 (v).  grad_out: device
 * [FS_PPO_ACTOR_PARAMS + FS_PPO_CRITIC_PARAMS] f32, each network's gradient in torch
 * parameters() order (w1, b1, w2, b2, w3, b3), as autograd defines it (torch.min
 * splits a tie's gradient, clamp passes it inside its closed range); loss_out: device
 * [3] f32 = the three means (policy, value, entropy).  Summation order is fixed, so
 * repeated calls give identical results. */
/* The update's forward passes without gradient, fp32, asynchronously on `stream`: for
 * x = device [n_values][8] f32 features, values_out[i] = critic(x[i]) for i < n_values, and
 * logp_out[i] = log_softmax(actor(x[i]))[actions[i]] for i < n_logp <= n_values (actions:
 * device uint8 [n_logp]).  Either output may be NULL (its network is then not run). */
int fs_ppo_eval(const float* x, int64_t n_values, const uint8_t* actions, int64_t n_logp, const fs_mlp* actor,
                const fs_mlp* critic, float* values_out, float* logp_out, void* stream);
int fs_ppo_grad(const float* rows, int64_t n, const fs_mlp* actor, const fs_mlp* critic, float clip,
                float vf_coef, float ent_coef, float* grad_out, float* loss_out, void* workspace,
                size_t workspace_bytes, void* stream);
/* The same two calls with the precision of the three 64-wide products (layer 2's forward pass,
 * the backward pass through W2 and dW2) chosen: FS_PPO_FP32 (fs_ppo_grad / fs_ppo_eval: fp32
 * MFMA, exact fp32 products) or FS_PPO_SPLIT_BF16 (each fp32 operand split into a bf16 hi + lo
 * pair and the product taken as hi.hi + hi.lo + lo.hi on bf16 MFMA with fp32 accumulation:
 * relative error per product below 2^-15, ~5x less matrix-pipe time).  The layers with 8 inputs
 * or outputs stay fp32; FS_PPO_SPLIT_BF16 takes tanh and exp from the hardware exp2 / reciprocal
 * (tanh within 2.5e-7 absolutely).  fs_ppo_eval_ex needs the workspace for FS_PPO_SPLIT_BF16 (NULL / 0
 * for FS_PPO_FP32); a workspace is not shared between calls in flight on different streams. */
#define FS_PPO_FP32 0
#define FS_PPO_SPLIT_BF16 1
int fs_ppo_grad_ex(const float* rows, int64_t n, const fs_mlp* actor, const fs_mlp* critic, float clip,
                   float vf_coef, float ent_coef, float* grad_out, float* loss_out, void* workspace,
                   size_t workspace_bytes, void* stream, int precision);
int fs_ppo_eval_ex(const float* x, int64_t n_values, const uint8_t* actions, int64_t n_logp, const fs_mlp* actor,
                   const fs_mlp* critic, float* values_out, float* logp_out, void* workspace, size_t workspace_bytes,
                   void* stream, int precision);
/* fs_ppo_grad_ex over a minibatch of whole runs of the [n_rows][12] table, without gathering it
 * first (ppo.py PPOTrainer.update: runs of consecutive samples in a shuffled order): sample i of
 * the minibatch is row runs[i >> run_shift] * 2^run_shift + (i mod 2^run_shift), for
 * i < n_runs * 2^run_shift; runs: device int64 [n_runs].  Same results, bit for bit, as
 * fs_ppo_grad_ex on those rows gathered in that order.  A run entry whose rows fall outside the
 * table is read as a padding row (nothing read, nothing added; the mean still counts it): the
 * entries are device data, so they are not checked on the host.  (ABI 6.) */
int fs_ppo_grad_runs(const float* rows, int64_t n_rows, const int64_t* runs, int64_t n_runs, int run_shift,
                     const fs_mlp* actor, const fs_mlp* critic, float clip, float vf_coef, float ent_coef,
                     float* grad_out, float* loss_out, void* workspace, size_t workspace_bytes, void* stream,
                     int precision);
/* GAE of a [T][N] trajectory (ppo.py gae), asynchronously on `stream`: rewards device
 * [T][N] f64 and done device [T][N] u8 as fs_step_n_policy's trajectory holds them, values
 * device [T + 1][N] f32 (the last row bootstraps); delta = (r + (gamma v[t+1]) keep) - v[t],
 * keep = 1 - done, adv[t] = delta[t] + gamma_lam keep[t] adv[t + 1] (one fused multiply-add),
 * ret = adv + v[t].  gamma and gamma_lam (= gamma * lam) as the f32 values torch rounds them to. */
int fs_ppo_gae(const double* rewards, const uint8_t* done, const float* values, int T, int64_t N, float gamma,
               float gamma_lam, float* adv_out, float* ret_out, void* stream);
/* The learner's features of n observations, asynchronously on `stream`: out device [n][8] f32
 * (16-byte aligned) = guard / 3, move / 16, move_frame / 55, position / 4.6 of both fighters
 * (wrappers/normalization.py's constants), each x * f32(1 / divisor in f64) as torch computes it; inputs are
 * trajectory columns ([n][2] u8, u8, f32, f32). */
int fs_ppo_features(const uint8_t* guard, const uint8_t* move, const float* move_frame, const float* position,
                    int64_t n, float* out, void* stream);
/* fs_ppo_grad's [n][12] row table from its columns, asynchronously on `stream`: x device
 * [n][8] f32 (16-byte aligned), actions u8 [n], old log-probs, advantages and returns f32 [n],
 * stats device [2] f32 = (mean, std) of the advantages; row = x, action,
 * old, (adv - mean) / (std + 1e-8), ret. */
int fs_ppo_pack(const float* x, const uint8_t* actions, const float* old_logp, const float* adv, const float* ret,
                const float* stats, int64_t n, float* rows_out, void* stream);

/* Fill device arrays p1_out/p2_out [n_steps][N] with the synthetic action stream
 * of fs_step_n (splitmix64 hash of (seed, arena_base + i, t0 + k, player)),
 * so benchmark inputs are resident in HBM before the timed region.
 * p2_out may be NULL. */
int fs_hash_actions(fs_handle h, int n_steps, uint64_t seed, uint64_t t0, uint8_t* p1_out, uint8_t* p2_out);

/* Device pointers of the current outputs, valid until the next call on h. */
int fs_outputs_get(fs_handle h, fs_outputs* out);

/* The host arrays of one FootsiesVectorEnv numpy step (vector_env.step_result_from_outputs, the
 * batched form of FE:336-380's _extract_obs / _extract_info and FE:555-570), in the reference's
 * dtypes: Gymnasium's MultiDiscrete as int64, Box as float32, bools as 0 / 1 bytes.  Any member
 * may be NULL (not written).  [N][2] arrays are P1, P2 per row; *_action are [N][3] (Left, Right,
 * Attack; state.py:26-36). */
typedef struct fs_host_arrays {
  int64_t* guard;            /* obs["guard"]      [N][2] */
  int64_t* move;             /* obs["move"]       [N][2] */
  float* move_frame;         /* obs["move_frame"] [N][2] */
  float* position;           /* obs["position"]   [N][2] */
  int64_t* info_guard;       /* the info's copies of the observation (FE:379) */
  int64_t* info_move;
  float* info_move_frame;
  float* info_position;
  int64_t* frame;            /* info["frame"]      [N] */
  uint8_t* p1_action;        /* info["p1_action"]  [N][3] bool */
  uint8_t* p2_action;        /* info["p2_action"]  [N][3] bool */
  int64_t* p1_hitstun;       /* info["p1_hitstun"] [N] */
  int64_t* p2_hitstun;       /* info["p2_hitstun"] [N] */
  double* reward;            /* [N] */
  uint8_t* terminated;       /* [N] bool */
  uint8_t* truncated;        /* [N] bool */
} fs_host_arrays;

/* Convert host copies of step outputs (`src`: the fs_outputs layout in host memory, e.g. the
 * pinned copy of fs_outputs_get's buffers, `n_src` rows each; only its first ten members are
 * read) into `dst`, over `threads` host threads (a pool kept by the library).  Row i of dst is
 * row rows[i] of src (rows NULL: row i), for i < n -- so the terminal records of the arenas that
 * ended a step are converted by passing the final_* arrays as src's first members and the
 * terminated rows.  FS_E_INVALID (nothing written) when a row index is outside [0, n_src) or,
 * without rows, n > n_src.  (ABI 5 added n_src.) */
int fs_host_convert(const fs_outputs* src, int64_t n_src, const int64_t* rows, int64_t n, const fs_host_arrays* dst,
                    int threads);
/* fs_host_convert started on the library's own threads, returning once its arguments are checked
 * (the same checks and errors); fs_host_convert_wait returns when it has finished.  The caller
 * goes on meanwhile -- FootsiesVectorEnv.step builds the terminated arenas' final-observation
 * dicts (Python, holding the GIL) while the step's arrays are converted -- and keeps src, rows and
 * dst valid until the wait.  One conversion in flight per process: a start while another (another
 * thread's) is in flight waits for it first; a wait returns once none is in flight.  fs_host_convert
 * calls for fewer than 8192 rows run on the calling thread and may overlap it.  (ABI 6.) */
int fs_host_convert_start(const fs_outputs* src, int64_t n_src, const int64_t* rows, int64_t n,
                          const fs_host_arrays* dst, int threads);
int fs_host_convert_wait(void);

/* Pack the current outputs into one FS_RECORD_BYTES record per arena at dst (device,
 * [N][40] bytes): guard[2] move[2] action[2] hitstun[2] u8, terminated u8, truncated
 * u8, pad[2], move_frame[2] f32, position[2] f32, frame i32, reward f64 -- the payload
 * of the multi-GPU per-step gather over RCCL.  Asynchronous. */
#define FS_RECORD_BYTES 40
int fs_pack_outputs(fs_handle h, void* dst);
/* fs_step that also writes every arena's FS_RECORD_BYTES record (fs_pack_outputs' layout) to rec
 * (device, [N][40] bytes, 8-byte aligned) from inside the tick's own kernel: the same bytes as
 * fs_step followed by fs_pack_outputs(h, rec), one launch instead of two -- the per-step gather
 * path of SURVEY.md 8(e).  With frame_delay > 0 (the delayed queue rewrites the outputs after the
 * tick) it is exactly those two calls.  Asynchronous.  (ABI 6.) */
int fs_step_rec(fs_handle h, const uint8_t* p1_act, const uint8_t* p2_act, int flags, void* rec);

/* Redirect the per-step outputs into caller-owned device buffers (e.g. torch
 * tensors) for zero-copy; NULL members keep the library's own buffer.  The
 * buffers must stay alive until fs_destroy or the next bind. */
int fs_bind_outputs(fs_handle h, const fs_outputs* dev);

/* Copy the raw EnvironmentState [N] / canonical full state [N] of every arena
 * to host memory (synchronous).  fs_get_state replaces STATE_SAVE
 * (BC:148-151, 667-674) in canonical form. */
int fs_get_env_state(fs_handle h, fs_env_state* host_out);
int fs_get_state(fs_handle h, fs_arena_state* host_out);
/* Load canonical state [N] from host (STATE_LOAD, BC:153-156, 676-683).
 * Input history beyond what fs_arena_state carries is not representable.  Fighters with
 * position_y != 0 or facing_flipped switch the handle's steps to the kernels' general-geometry
 * path (box y extents tested, y carried through the pushes) until the next fs_set_state loads
 * only standard fighters.
 * FS_E_INVALID (nothing loaded) for a field outside the packed layout's range, or, with the
 * bot as P2, a queue index at or past its plan's length (such a queue is empty: plan -1). */
int fs_set_state(fs_handle h, const fs_arena_state* host_in);

/* Block until all work on the handle's stream is done. */
int fs_sync(fs_handle h);
/* The handle's hipStream_t (as void*), for event timing / torch.cuda.ExternalStream. */
void* fs_stream(fs_handle h);
/* Run all further work of h on a caller-owned hipStream_t (e.g. PyTorch's current
 * stream; NULL = the HIP null stream) instead of the library's own, so device
 * actions/outputs are ordered with the caller's kernels without events.
 * FS_STREAM_OWN restores the library's stream.  The caller keeps the stream
 * alive while h uses it; switching orders the new stream after the old one. */
#define FS_STREAM_OWN ((void*)(intptr_t)-1)
int fs_set_stream(fs_handle h, void* stream);
int fs_num_envs(fs_handle h);
uint64_t fs_steps_taken(fs_handle h);
/* The kernel a step call on h would launch, as rocprofv3 names it ("fsk::k_step_n<0, 0>"):
 * n_steps = 1 is fs_step / fs_step_masked, n_steps > 1 fs_step_n with action rows (its launches
 * pick the one-lane kernel from 2 x 64 x SIMD-count arenas on, FOOTSIES_FUSED_LANES forces
 * either); flags FS_KERNEL_HASHED = fs_step_n without action rows, FS_KERNEL_POLICY =
 * fs_step_n_policy, FS_KERNEL_PACKED = fs_step_n_packed.  For naming profiles and roofline lines; NULL for a bad handle or flags.
 * The string stays valid until the calling thread's next call. */
#define FS_KERNEL_HASHED 1
#define FS_KERNEL_POLICY 2
#define FS_KERNEL_PACKED 4  /* fs_step_n_packed */
const char* fs_step_kernel(fs_handle h, int n_steps, int flags);
void fs_destroy(fs_handle h);
/* Last error message of h (or of the last failed fs_create when h is NULL). */
const char* fs_last_error(fs_handle h);

#ifdef __cplusplus
}
#endif
#endif /* FOOTSIES_H */
