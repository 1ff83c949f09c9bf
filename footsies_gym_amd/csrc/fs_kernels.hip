// fs_kernels.hip -- HIP kernels for gfx950 (MI355X): the FOOTSIES Fight tick for N arenas.
//
// A Fight tick of the reference (BattleCore.FixedUpdate Fight branch ->
// UpdateFightState, Assets/Script/BattleCore.cs:201-220, 347-364) is restated
// over a bit-packed, struct-of-arrays arena state in HBM, two lanes per arena
// (one fighter each, partner values exchanged with DPP):
//
//   load (coalesced 4/8/16-B per lane) -> n ticks in registers -> store
//
// Frame data is one 31 KB image (fs_tables.h), staged into LDS per block by the fused launches
// and read in place from global memory by the one-tick launch: per action a 16-B ActionInfo
// (frame count, loop, cancel window), per (action, frame) an index into 53 de-duplicated frame
// records (three 16-B entries of x geometry and velocity) -- the window scans of
// ActionData.cs:87-168 resolved offline (tools/gen_tables.py) -- the request chain's outcome per
// (action, window state, inputs), the box-pair y overlaps per record pair and the hit resolution
// per (attacker hit count, attacker record).  A tick's dependent LDS round trips: action info
// (issued after the previous tick's collision), then the record index and the request-table
// entry together, then the frame record with the y-overlap bits and the resolution entry.  The
// 180-deep input histories
// (Fighter.cs:98-101) are two 16-frame shift registers (backward / forward relative to the
// fighter's facing) plus a saturating attack-hold counter: the reference
// only reads input[0..16] for dashes (Fighter.cs:585-635, dashAllowFrame 9) and
// "attack held on input[1..59]" for the charge special (Fighter.cs:569-583).
//
// Float arithmetic follows the C# expression order with every binary32
// operation rounded (__fadd_rn/__fmul_rn; the file is also built with
// -ffp-contract=off) or, in FS_FLOAT_DOUBLE mode, with binary64 temporaries.
//
// Paths: BC = Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs,
// AI = Assets/Script/BattleAI.cs, FE = footsies-gym/footsies_gym/envs/footsies.py.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "fs_internal.h"
#include "fs_tables.h"
#include "fs_policy.h"

#pragma clang fp contract(off)

namespace fsk {

constexpr int NONE = 31;  // empty buffer / reserve slot
constexpr uint32_t IN_LEFT = 1, IN_RIGHT = 2, IN_ATTACK = 4;

// ---------------------------------------------------------------------------
// frame data staged in LDS.  Every lookup of the tick (action info -> record index and
// request entry -> frame record) is a dependent, lane-divergent load; from LDS it costs
// ~tens of cycles instead of an L1/L2 round trip.  31 KB per block, copied once per fused
// launch by all threads of the block.
// ---------------------------------------------------------------------------
__shared__ Tables sT;

constexpr int kBlock = 256;

// Where a kernel reads the tables from: G = false, the LDS image every block stages (sT, sBot);
// G = true, the __constant__ images in global memory through the vector L1 / L2 (kTables, kBot).
// The fused launches stage (one copy serves hundreds of ticks); a one-tick launch (k_step) reads
// them in place, which costs less than staging the image in every block for a single tick.
template <bool G>
__device__ __forceinline__ const Tables& tabs() {
  if constexpr (G) return kTables;
  else return sT;
}
// Table placement of a launch (env_step's TP): all in LDS (the fused launches) or all in
// global memory (k_step).  Measured alike for k_step: staging every table but the 17 KB request
// table (13.5 KB per block) so that one dependent read per tick goes to L2 instead of three.
constexpr int kTabLds = 0, kTabGlobal = 1;

// ---------------------------------------------------------------------------
// packed fighter word (u64), one per fighter in DevState::fpk
//   [0,5) action idx | [5,14) action frame | [14,19) hitstun | [19,21) vital |
//   [21,23) guard | [23,25) hit count | [25,30) buffer idx | [30,35) reserve idx |
//   35 isInputBackward | 36 isReserveProximityGuard | 37 hasWon | [38,44) attack hold |
//   44 facing flipped (isFaceRight != isPlayerOne, only after a state load)
// arena header word (DevState::aw.y)
//   [0,15) recording count | [15,18) rec P1 | [18,21) rec P2 | [21,24) remote actor P1 input |
//   [24,27) remote actor P2 input | 27 reset pending | 28 has_terminated | 29 P2's actor is the bot
// bot word (DevState::bot.x for P2's BattleAI, DevState::bot1.x for P1's)
//   [0,3) move plan+1 (0 = empty) | [3,10) move index | [10,13) attack plan+1 |
//   [13,20) attack index | [20,25) previous FightState opponent action idx |
//   25 ready (fightStates[5] set) | [26,29) the bot actor's last input (TrainingBattleAIActor.input)
// ---------------------------------------------------------------------------

// A pair of like box values (the x of box 0 and 1, or their half-widths): <2 x float> arithmetic is
// one packed instruction (v_pk_add_f32), each half rounded exactly as the scalar op.
typedef float F2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ F2 splat(float v) { return F2{v, v}; }

struct Fighter {
  float x;
  uint32_t hist;  // input[0..15]: bit j = backward on input[j], bit 16 + j = forward (see split_hist)
  int act, frame, stun, vital, guard, hits, buf, rsv, hold;
  uint32_t in_back, prox, won;  // flags as 0 / 1 words (a carried bool is re-masked at every test)
  // boxes of this tick (UpdateBoxes, F:671-697): the frame record holds their geometry,
  // the fighter their world x (y == rect.y while position.y is 0)
  int rec;        // frame record index of (action, frame)
  float px, ux0, ux1, hx0, hx1;  // world x: pushbox, hurtbox 0 / 1, hitbox 0 / 1
  float pw, phw;  // pushbox width of the record, and width / 2
  // General geometry (a launch with StepParams::geom; otherwise flip == 0 and y == 0 throughout):
  uint32_t flip;  // isFaceRight != isPlayerOne (LoadState F:744; SetupBattleStart F:124 clears it)
  float y;        // position.y
  float py, uy0, uy1, hy0, hy1;  // world y (rect.y) of the pushbox, hurtboxes 0 / 1, hitboxes 0 / 1
};

struct Arena {
  Fighter f0, f1;
  int frame_count;
  uint32_t rec_count, rec1, rec2, act1, act2;
  bool pending, has_term;
  double cum;
  uint4 rng;
  bool p2bot;
  uint2 bw[2];  // bot words of P1's and P2's BattleAI (decoded by the state kernels)
};

__device__ __forceinline__ void unpack_fighter(Fighter& f, uint32_t lo, uint32_t hi) {
  uint64_t w = ((uint64_t)hi << 32) | lo;
  f.act = (int)(w & 31);
  f.frame = (int)((w >> 5) & 511);
  f.stun = (int)((w >> 14) & 31);
  f.vital = (int)((w >> 19) & 3);
  f.guard = (int)((w >> 21) & 3);
  f.hits = (int)((w >> 23) & 3);
  f.buf = (int)((w >> 25) & 31);
  f.rsv = (int)((w >> 30) & 31);
  f.in_back = (w >> 35) & 1;
  f.prox = (w >> 36) & 1;
  f.won = (w >> 37) & 1;
  f.hold = (int)((w >> 38) & 63);
  f.flip = (w >> 44) & 1;
}

__device__ __forceinline__ uint64_t pack_fighter(const Fighter& f) {
  return (uint64_t)f.act | ((uint64_t)f.frame << 5) | ((uint64_t)f.stun << 14) | ((uint64_t)f.vital << 19) |
         ((uint64_t)f.guard << 21) | ((uint64_t)f.hits << 23) | ((uint64_t)f.buf << 25) |
         ((uint64_t)f.rsv << 30) | ((uint64_t)f.in_back << 35) | ((uint64_t)f.prox << 36) |
         ((uint64_t)f.won << 37) | ((uint64_t)f.hold << 38) | ((uint64_t)f.flip << 44);
}

__device__ __forceinline__ void load_arena(Arena& A, const DevState& s, int i) {
  float2 pos = s.pos[i];
  uint2 hist = s.hist[i];
  uint4 pk = s.fpk[i];
  int2 aw = s.aw[i];
  A.cum = s.cum[i];
  unpack_fighter(A.f0, pk.x, pk.y);
  unpack_fighter(A.f1, pk.z, pk.w);
  A.f0.x = pos.x;
  A.f1.x = pos.y;
  const float2 py = s.posy[i];
  A.f0.y = py.x;
  A.f1.y = py.y;
  A.f0.hist = hist.x;  // split form (get/set convert)
  A.f1.hist = hist.y;
  A.frame_count = aw.x;
  uint32_t h = (uint32_t)aw.y;
  A.rec_count = h & 0x7fff;
  A.rec1 = (h >> 15) & 7;
  A.rec2 = (h >> 18) & 7;
  A.act1 = (h >> 21) & 7;
  A.act2 = (h >> 24) & 7;
  A.pending = (h >> 27) & 1;
  A.has_term = (h >> 28) & 1;
  A.p2bot = (h >> 29) & 1;
  A.rng = s.rng[i];
  A.bw[0] = s.bot1[i];
  A.bw[1] = s.bot[i];
}

__device__ __forceinline__ void store_arena(const Arena& A, const DevState& s, int i) {
  uint64_t w0 = pack_fighter(A.f0), w1 = pack_fighter(A.f1);
  s.pos[i] = make_float2(A.f0.x, A.f1.x);
  s.posy[i] = make_float2(A.f0.y, A.f1.y);
  s.hist[i] = make_uint2(A.f0.hist, A.f1.hist);
  s.fpk[i] = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
  uint32_t h = A.rec_count | (A.rec1 << 15) | (A.rec2 << 18) | (A.act1 << 21) | (A.act2 << 24) |
               ((uint32_t)A.pending << 27) | ((uint32_t)A.has_term << 28) | ((uint32_t)A.p2bot << 29);
  s.aw[i] = make_int2(A.frame_count, (int)h);
  s.cum[i] = A.cum;
  s.rng[i] = A.rng;
  s.bot1[i] = A.bw[0];
  s.bot[i] = A.bw[1];
}

// ---------------------------------------------------------------------------
// float expression model (see oracle/footsies_oracle.c for the same forms)
// ---------------------------------------------------------------------------
template <int FM>
__device__ __forceinline__ float fadd(float a, float b) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return (float)__dadd_rn((double)a, (double)b);
  else return __fadd_rn(a, b);
}
template <int FM>
__device__ __forceinline__ float fsub(float a, float b) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return (float)__dsub_rn((double)a, (double)b);
  else return __fsub_rn(a, b);
}
template <int FM>
__device__ __forceinline__ F2 fadd2(F2 a, F2 b) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return F2{fadd<FM>(a.x, b.x), fadd<FM>(a.y, b.y)};
  else return a + b;  // (-ffp-contract=off: nothing fuses into it)
}
template <int FM>
__device__ __forceinline__ F2 fsub2(F2 a, F2 b) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return F2{fsub<FM>(a.x, b.x), fsub<FM>(a.y, b.y)};
  else return a - b;
}
// ---------------------------------------------------------------------------
// input (F:172-188, 569-666)
// ---------------------------------------------------------------------------
// The inputs UpdateActionRequest reads, as small integer codes (the request table's index
// fields) computed with bit arithmetic in VGPRs rather than as compare-and-select booleans.
struct InputEval {
  uint32_t held;  // bit 0 = backward held on input[0], bit 1 = forward (facing-relative)
  uint32_t atk;   // 1 = special (attack released after the charge), 2 = attack pressed, else 0
  uint32_t dash;  // 1 = forward dash, 2 = backward dash, else 0
};

// Left/Right -> (bit0 = backward, bit1 = forward).  P1 faces right, P2 left for
// the whole match (SetupBattleStart, F:124; BC:264-265).
__device__ __forceinline__ uint32_t rel_bits(uint32_t in, int k) {
  in &= 3;
  return k == 0 ? in : (((in & 1) << 1) | (in >> 1));
}
__device__ __forceinline__ uint32_t compact_even(uint32_t x) {
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0F0F0F0Fu;
  x = (x | (x >> 4)) & 0x00FF00FFu;
  x = (x | (x >> 8)) & 0x0000FFFFu;
  return x;
}
__device__ __forceinline__ uint32_t spread_even(uint32_t x) {
  x &= 0x0000FFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}
// The state API's history is raw Left/Right bit pairs per frame (input[j] at bits
// 2j, 2j+1); the kernels keep the facing-relative split form, so a tick shifts two
// registers at once and the dash parsers read them directly.
__device__ __forceinline__ uint32_t split_hist(uint32_t raw, int k) {
  const uint32_t rel = k == 0 ? raw : (((raw & 0x55555555u) << 1) | ((raw >> 1) & 0x55555555u));
  return compact_even(rel) | (compact_even(rel >> 1) << 16);
}
__device__ __forceinline__ uint32_t raw_hist(uint32_t h, int k) {
  const uint32_t b = spread_even(h), f = spread_even(h >> 16);
  return k == 0 ? (b | (f << 1)) : (f | (b << 1));
}

// rel_bits as a per-lane table: entry `in` (2 bits at 2 in, for in = 0..7) of kRelLut[k], so a tick
// spends one bit-field extract on it (the select of the lane's table is loop-invariant)
constexpr uint32_t kRelLut0 = 0xE4E4u, kRelLut1 = 0xD8D8u;  // 3,2,1,0 / 3,1,2,0 per 4 inputs

// UpdateInput + the reads UpdateActionRequest makes of the new history.  rlut = kRelLut0 / kRelLut1
// for P1 / P2.
__device__ __forceinline__ InputEval update_input(Fighter& f, uint32_t in, uint32_t rlut) {
  const uint32_t old_hist = f.hist;
  const int old_hold = f.hold;
  const uint32_t r0 = __builtin_amdgcn_ubfe(rlut, in << 1, 2);  // == rel_bits(in, k)
  f.hist = ((old_hist << 1) & 0xFFFEFFFEu) | (r0 & 1) | ((r0 & 2) << 15);
  f.hold = (in & IN_ATTACK) ? min(old_hold + 1, 63) : 0;
  InputEval e;
  e.held = r0;
  // inputDown[0] & Attack with input[1] released; inputUp[0] & Attack after input[1..59] held
  const uint32_t atk_now = (in >> 2) & 1u;
  const uint32_t held_long = ((uint32_t)(old_hold - (kSpecialHoldFrame - 1)) >> 31) ^ 1u;  // old_hold >= 59
  const uint32_t was_up = (uint32_t)(old_hold - 1) >> 31;                                  // old_hold == 0
  e.atk = (held_long & ~atk_now & 1u) | ((atk_now & was_up) << 1);
  // dash parsers over input[1..16] (bit j-1 of each mask = input[j]): j = the first input among
  // input[1..8] with a direction (8 when none); masking F and B to that window makes isF = isB = 0
  // when there is none, so no separate "found" test is needed
  const uint32_t B = old_hist & 0xFFFFu, F = old_hist >> 16, E = B | F;
  const uint32_t win = (1u << (kDashAllowFrame - 1)) - 1u;
  const uint32_t j = (uint32_t)__builtin_ctz((E & win) | (1u << (kDashAllowFrame - 1)));
  const uint32_t neutral = min((~E >> (j + 1)) & win, 1u);  // some input[j+2 .. j+9] with neither direction
  const uint32_t isF = ((F & win) >> j) & 1u, isB = ((B & win) >> j) & 1u;
  const uint32_t fd = isF & ~isB & neutral & (r0 >> 1) & ~F;  // forward now, not on input[1]
  const uint32_t bd = isB & ~isF & neutral & r0 & ~B;         // backward now, not on input[1]
  e.dash = (fd & 1u) | ((bd & 1u) << 1);
  return e;
}

// ---------------------------------------------------------------------------
// action state machine (F:140-166, 201-286, 472-510, 546-563)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void set_action(Fighter& f, int a) {  // SetCurrentAction (F:546-563)
  f.act = a;
  f.frame = 0;
  f.hits = 0;
  f.buf = NONE;
  f.rsv = NONE;
}

// ActionInfo (fs_tables.h) travels in registers as its raw 16 bytes: selecting
// between two struct values (HIP's uint4 included) would go through scratch memory.
typedef uint32_t AInfo __attribute__((ext_vector_type(4)));  // a native vector: selects stay in registers
template <bool G>
__device__ __forceinline__ AInfo action_info(int a) { return reinterpret_cast<const AInfo*>(tabs<G>().action)[a]; }
__device__ __forceinline__ AInfo stand_info() {  // action_info(A_STAND), as constants
  AInfo i;
  i.x = kStandInfo[0];
  i.y = kStandInfo[1];
  i.z = kStandInfo[2];
  i.w = kStandInfo[3];
  return i;
}
__device__ __forceinline__ int ai_frame_count(AInfo i) { return (int)(int16_t)(i.x & 0xffffu); }
__device__ __forceinline__ int ai_loop_from(AInfo i) { return (int)(int16_t)(i.x >> 16); }
__device__ __forceinline__ bool ai_always_cancel(AInfo i) { return (i.y & 0xffu) != 0; }
__device__ __forceinline__ int ai_cancel_lo(AInfo i) { return (int)((i.y >> 16) & 0xffu); }
__device__ __forceinline__ int ai_cancel_hi(AInfo i) { return (int)(i.y >> 24); }
__device__ __forceinline__ uint32_t ai_cancel_mask(AInfo i) { return i.z; }
static_assert(sizeof(ActionInfo) == 16, "ActionInfo must be 16 bytes");

// IncrementActionFrame (F:140-166); `ai` = ActionInfo of f.act
__device__ __forceinline__ void increment_action_frame(Fighter& f, AInfo ai) {
  const bool stunned = f.stun > 0;
  f.stun -= stunned ? 1 : 0;
  const int next = f.frame + 1;
  const int loop_from = ai_loop_from(ai);
  const int looped = (next >= ai_frame_count(ai) && loop_from >= 0) ? loop_from : next;
  f.frame = stunned ? f.frame : looped;
}

// UpdateActionRequest (F:201-286) as one read of kTables.req_table (tools/gen_tables.py runs
// RequestAction's chain, F:472-510, offline for every case), branch-free:
// * hasWon (F:204-208; set only between KO and the next SetupBattleStart, or by STATE_LOAD):
//   RequestAction(WIN) against the current action's take / buffer masks, entry kReqWin + 3 act + cls;
// * the reserved damage action, then the buffered cancel (F:212-229): SetCurrentAction(a0),
//   entry kReqEarly + a0;
// * otherwise the request chain (special / attack F:234-254, dash F:256-259, movement F:265-283):
//   its outcome depends only on the action, whether it has ended or sits in its cancel window,
//   the attack / dash / held direction inputs and the proximity latch.
// The first two return before the latches are touched (F:263, 285).  Returns whether
// SetCurrentAction ran; then *rec is the new action's frame-0 record.
// The request table entry a fighter reads this tick (`keep`: hasWon or an early return, which
// leave the guard latches alone) ...
__device__ __forceinline__ uint32_t request_sel(const Fighter& f, const InputEval& e, AInfo ai, bool& keep) {
  // (take_rsv = rsv set & no stun; take_buf = !take_rsv & buf set & (hit or whiff-cancel) & no stun,
  // as bitwise ops: the short-circuit form materializes each condition as a 0 / 1 word)
  const int rsv = f.rsv, buf = f.buf;
  const bool has_rsv = rsv != NONE;
  const bool won = f.won != 0;
  const bool early = (f.stun <= 0) & (has_rsv | ((buf != NONE) & (kCanCancelOnWhiff | (f.hits > 0))));
  const int a0 = has_rsv ? rsv : buf;
  const bool ended = f.frame >= ai_frame_count(ai);
  const bool inwin = (f.frame >= ai_cancel_lo(ai)) & (f.frame <= ai_cancel_hi(ai));
  const uint32_t cls = ended ? 2u : (inwin ? 1u : 0u);
  // (the low five bits XOR-swizzled with the action, as tools/gen_tables.py lays the table out:
  // lanes that differ in action but not in inputs read different LDS banks)
  const uint32_t in8 = ((9u * cls + 3u * e.atk + e.dash) << 3) | (e.held << 1) | (uint32_t)f.prox;
  const uint32_t idx = ((uint32_t)f.act << 8) | (in8 ^ (uint32_t)f.act);
  keep = early | won;
  return won ? (uint32_t)kReqWin + 3u * (uint32_t)f.act + cls : (early ? (uint32_t)(kReqEarly + a0) : idx);
}
// ... and what the entry q does to it.  Returns whether SetCurrentAction ran; then *rec is the new
// action's frame-0 record.
__device__ __forceinline__ bool apply_request(Fighter& f, uint32_t q, bool keep, const InputEval& e, uint32_t* rec) {
  const bool set = ((q >> 11) & 1u) != 0;  // SetCurrentAction ran (F:546-563)
  const bool bset = ((q >> 10) & 1u) != 0;
  f.act = set ? (int)(q & 31u) : f.act;
  f.buf = set ? NONE : (bset ? (int)((q >> 5) & 31u) : f.buf);
  f.frame = set ? 0 : f.frame;
  f.hits = set ? 0 : f.hits;
  f.rsv = set ? NONE : f.rsv;
  f.in_back = keep ? f.in_back : (e.held & 1u);  // for proximity guard (F:263)
  f.prox = keep ? f.prox : 0u;                   // F:285
  *rec = (q >> 12) & 255u;
  return set;
}
template <bool G>
__device__ __forceinline__ bool update_action_request(Fighter& f, const InputEval& e, AInfo ai, uint32_t* rec) {
  bool keep;
  const uint32_t sel = request_sel(f, e, ai, keep);
  return apply_request(f, tabs<G>().req_table[sel], keep, e, rec);
}

// UpdateMovement (F:291-319).  FORWARD / BACKWARD walk at the fighter speeds, any other action
// takes the first movement window's velocity (0 = none).  BACKWARD's `pos -= s*sign*dt` is
// `pos + (-s)*sign*dt` bit for bit (negation is exact and round-to-nearest is symmetric), and
// `v*sign` is exact too, so every case is pos + v*dt with v pre-signed in the frame record:
// tools/gen_tables.py stores the walk speeds in the FORWARD / BACKWARD records.
template <int FM>
__device__ __forceinline__ void update_movement(Fighter& f, float v) {
  float nx;
  if constexpr (FM == FS_FLOAT_DOUBLE) nx = (float)__dadd_rn((double)f.x, __dmul_rn((double)v, (double)kDt));
  else nx = __fadd_rn(f.x, __fmul_rn(v, kDt));
  f.x = (f.stun <= 0 && v != 0.0f) ? nx : f.x;
}

// The frame record `rec` of facing `k` in LDS (fs_tables.h: rec_push / rec_hurt / rec_hit, one
// 16-B entry each).  The byte offset is formed with 24-bit multiplies (v_mul_u32_u24, full rate):
// indexing the arrays directly makes a 64-bit v_mad_u64_u32 and a v_mul_lo_u32, both quarter-rate,
// on the dependency chain of every tick.
typedef float F4 __attribute__((ext_vector_type(4)));     // native vectors: they stay in registers
typedef uint32_t U4 __attribute__((ext_vector_type(4)));
struct RecGeo {
  F4 push;  // pushbox x offset, width, velocity, width / 2
  F4 hurt;  // hurtbox 0 / 1 x offsets, hurtbox 0 / 1 width / 2 (.xy / .zw: packed-f32 pairs)
  F4 hit;   // hitbox 0 / 1 x offsets, hitbox 0 / 1 width / 2
};
template <bool G>
__device__ __forceinline__ RecGeo frame_rec(uint32_t k, uint32_t rec) {
  const Tables& T = tabs<G>();
  const uint32_t off = __umul24(k, (uint32_t)sizeof(T.rec_push[0])) + (rec << 4);  // rec < 64
  auto at = [&](const void* base) {
    return *reinterpret_cast<const F4*>(reinterpret_cast<const char*>(base) + off);
  };
  RecGeo g;
  g.push = at(&T.rec_push[0][0]);
  g.hurt = at(&T.rec_hurt[0][0]);
  g.hit = at(&T.rec_hit[0][0]);
  return g;
}

// the frame record of (act, frame)
template <bool G>
__device__ __forceinline__ int frame_record(const Fighter& f) {
  return tabs<G>().rec_index[f.act * kFrameStride + min(f.frame, kFrameStride - 1)];
}

// UpdateBoxes (F:671-697): world x of every box of the record, `R` being the record in
// the fighter's facing (x offsets pre-signed): basePosition.x + dataRect.x * sign.
template <int FM>
__device__ __forceinline__ void update_boxes(Fighter& f, const RecGeo& R) {
  f.pw = R.push.y;
  f.phw = R.push.w;
  f.px = fadd<FM>(f.x, R.push.x);
  const F2 ux = fadd2<FM>(splat(f.x), R.hurt.xy), hx = fadd2<FM>(splat(f.x), R.hit.xy);
  f.ux0 = ux.x;
  f.ux1 = ux.y;
  f.hx0 = hx.x;
  f.hx1 = hx.y;
}

// ApplyPositionChange (F:331-350): position and every box are shifted, not rebuilt
template <int FM>
__device__ __forceinline__ void apply_position_change(Fighter& f, float dx) {
  const F2 xp = fadd2<FM>(F2{f.x, f.px}, splat(dx));
  f.x = xp.x;
  f.px = xp.y;
  const F2 ux = fadd2<FM>(F2{f.ux0, f.ux1}, splat(dx)), hx = fadd2<FM>(F2{f.hx0, f.hx1}, splat(dx));
  f.ux0 = ux.x;
  f.ux1 = ux.y;
  f.hx0 = hx.x;
  f.hx1 = hx.y;
}

// General geometry (StepParams::geom: some fighter was loaded with position.y != 0 or a flipped
// facing).  The box y extents come from kRecY (fs_tables.h) instead of ybits / the constant
// pushbox y-test, the world y of every box is position.y + rect.y (TransformToFightRect
// F:706-719), and the pushes carry position.y through ApplyPositionChange as the C# does: both
// UpdatePushCharacterVs* calls pass a fighter's position.y as the y shift (BC:491-498, 511-515),
// so every push adds y to itself (P2's shift in the P1-right-of-P2 case is P1's y after P1's own
// shift).  A fighter whose y is 0 gets the same results as on the standard path.
struct RecY {
  F4 a, b, c;  // {push y, h, hurt 0 y, h}, {hurt 1 y, h, hit 0 y, h}, {hit 1 y, h, -, -}
};
__device__ __forceinline__ RecY rec_y(uint32_t rec) {
  const F4* t = reinterpret_cast<const F4*>(kRecY);
  return RecY{t[3 * rec], t[3 * rec + 1], t[3 * rec + 2]};
}
template <int FM>
__device__ __forceinline__ void update_boxes_y(Fighter& f, const RecY& Y) {
  f.py = fadd<FM>(f.y, Y.a.x);
  f.uy0 = fadd<FM>(f.y, Y.a.z);
  f.uy1 = fadd<FM>(f.y, Y.b.x);
  f.hy0 = fadd<FM>(f.y, Y.b.z);
  f.hy1 = fadd<FM>(f.y, Y.c.x);
}
template <int FM>
__device__ __forceinline__ void apply_position_change_y(Fighter& f, float dy) {  // F:334-349, the y half
  f.y = fadd<FM>(f.y, dy);
  f.py = fadd<FM>(f.py, dy);
  f.uy0 = fadd<FM>(f.uy0, dy);
  f.uy1 = fadd<FM>(f.uy1, dy);
  f.hy0 = fadd<FM>(f.hy0, dy);
  f.hy1 = fadd<FM>(f.hy1, dy);
}

// UpdatePushCharacterVsBackground (BC:503-519) with BoxBase semantics
// Branch-free: with no push the shift is -0.0, the exact identity of IEEE addition (x + -0.0 == x
// bit for bit, -0.0 included), so every lane applies it.
template <int FM, bool GEOM = false>
__device__ __forceinline__ void push_character_vs_background(Fighter& f) {
  // BoxBase xMin / xMax (F:12-13) with the record's exact width / 2 (w / 2 is exact in binary32,
  // and (double)(w / 2) == (double)w / 2 for the binary64 model)
  // (xMin, xMax) as one pair: px - w/2 is px + (-w/2) bit for bit (IEEE subtraction is defined so)
  const float xmin = fsub<FM>(f.px, f.phw), xmax = fadd<FM>(f.px, f.phw);
  float d_lo = fsub<FM>(-kStageHalf, xmin), d_hi = fsub<FM>(kStageHalf, xmax);
  asm volatile("" : "+v"(d_lo), "+v"(d_hi));  // both computed: selects, not a branch
  const float dx = xmin < -kStageHalf ? d_lo : (xmax > kStageHalf ? d_hi : -0.0f);
  apply_position_change<FM>(f, dx);
  if constexpr (GEOM) {  // ApplyPositionChange(dx, f.position.y) on a push; x + -0.0 == x otherwise
    const bool pushed = (xmin < -kStageHalf) | (xmax > kStageHalf);
    apply_position_change_y<FM>(f, pushed ? f.y : -0.0f);
  }
}

// BoxBase (F:8-26): boxes are (world x, width/2, yMin, yMax); xMin = x - w/2, xMax = x + w/2
// (F:12-13) and Overlaps is inclusive.  The hit test below evaluates it per box pair.

constexpr int DR_DAMAGE = 1, DR_GUARD = 2, DR_GUARD_BREAK = 3;

// NotifyDamaged (F:357-398)
__device__ __forceinline__ int notify_damaged(Fighter& f, const AttackInfo& ad) {
  bool guard_break = false;
  if (ad.guard_damage > 0) {
    f.guard -= ad.guard_damage;
    if (f.guard < 0) {
      guard_break = true;
      f.guard = 0;
    }
  }
  if (f.act == A_BACKWARD || ((kGuardTypeMask >> f.act) & 1u)) {
    set_action(f, ad.guard_action);
    if (guard_break) {
      f.rsv = A_GUARD_BREAK;
      return DR_GUARD_BREAK;
    }
    return DR_GUARD;
  }
  if (ad.vital_damage > 0) {
    f.vital -= ad.vital_damage;
    if (f.vital <= 0) f.vital = 0;
  }
  set_action(f, ad.damage_action);
  return DR_DAMAGE;
}

// The box test of one attacker of UpdateHitboxHurtboxCollision (BC:535-569): the
// attacker's hitboxes in order, skipping attacks that already hit (CanAttackHit,
// F:408-420); a proximity box only flags proximity, a real box is a hit and ends
// the scan.  Branch-free over the 2x2 box pairs: the hit's attack is the first real
// box that overlaps, and proximity only matters when nothing hit.  The overlaps do
// not depend on the attacker's hit count, so they are computed once, as a 4-bit mask
// (bit 2j+i: attacker hitbox j overlaps defender hurtbox i); the resolution for every
// hit count is one entry of kTables.resolve per (attacker record, mask), generated
// offline (tools/gen_tables.py).
// The x half of BoxBase.Overlaps (F:17-25) per box pair, with each box's xMin / xMax computed
// once, as mask bits 2j+i.  The y half depends on the two frame records alone (boxes move in x
// only) and comes from kTables.ybits, which is also 0 for absent boxes (past a record's box
// count), so no count checks are needed here.
template <int FM>
__device__ __forceinline__ uint32_t box_x_overlaps(float hw0, float hw1, float hx0, float hx1, F2 uw, F2 ux) {
  const float h0min = fsub<FM>(hx0, hw0), h0max = fadd<FM>(hx0, hw0);
  const float h1min = fsub<FM>(hx1, hw1), h1max = fadd<FM>(hx1, hw1);
  const F2 umin = fsub2<FM>(ux, uw), umax = fadd2<FM>(ux, uw);  // my hurtboxes 0 / 1
  const float u0min = umin.x, u0max = umax.x, u1min = umin.y, u1max = umax.y;
  auto ov = [](float smin, float smax, float omin, float omax) {
    return (uint32_t)((omax >= smin) & (omin <= smax));
  };
  return ov(h0min, h0max, u0min, u0max) | (ov(h0min, h0max, u1min, u1max) << 1) |
         (ov(h1min, h1max, u0min, u0max) << 2) | (ov(h1min, h1max, u1min, u1max) << 3);
}

// ---------------------------------------------------------------------------
// bot: BattleAI for P2 (AI:10-403) with queues as (plan, index)
// ---------------------------------------------------------------------------
// (the plan enums and lengths are in fs_internal.h: fs_set_state validates queue indices with them)

__device__ __forceinline__ uint32_t rng_next(uint4& s) {  // UnityEngine.Random Xorshift128
  const uint32_t t = s.x ^ (s.x << 11);
  s.x = s.y;
  s.y = s.z;
  s.z = s.w;
  s.w = s.w ^ (s.w >> 19) ^ t ^ (t >> 8);
  return s.w;
}
// A select between two uint4 values, one component at a time.  HIP's uint4 is a struct: a `c ? a :
// b` on it is lowered through a private-memory copy and a dynamically addressed load (48-64 B of
// scratch per lane in the per-arena-actor kernels before this helper); four 32-bit selects stay in
// registers.
__device__ __forceinline__ uint4 sel4(bool c, const uint4& a, const uint4& b) {
  uint4 r;
  r.x = c ? a.x : b.x;
  r.y = c ? a.y : b.y;
  r.z = c ? a.z : b.z;
  r.w = c ? a.w : b.w;
  return r;
}
__device__ __forceinline__ uint4 rng_init(int32_t seed) {  // Random.InitState
  uint4 s;
  s.x = (uint32_t)seed;
  s.y = s.x * 1812433253u + 1u;
  s.z = s.y * 1812433253u + 1u;
  s.w = s.z * 1812433253u + 1u;
  return s;
}

// P2's forward is Left, backward is Right (AI:380-388); the dash plans are
// [F, 0, F] -- AddBackwardDashInputQueue also enqueues forward (AI:337-342).
constexpr uint32_t move_plan_input(uint32_t plan, uint32_t i) {
  const uint32_t F = IN_LEFT, B = IN_RIGHT;
  switch (plan) {
    case MP_FAR1: return i < 40 ? F : i < 50 ? B : i < 80 ? F : B;
    case MP_FAR2: {
      const uint32_t j = i < 28 ? i : i - 28;
      return j < 3 ? (j == 1 ? 0u : F) : B;
    }
    case MP_MID1: return i < 30 ? F : i < 40 ? B : i < 60 ? F : B;
    case MP_MID2:
    case MP_FALLBACK2: return i < 3 ? (i == 1 ? 0u : F) : B;
    case MP_FALLBACK1: return B;
    default: return 0u;  // MP_NEUTRAL
  }
}
// frames at the start of an attack plan with Attack held; AP_TWO_HIT also presses at index 4
constexpr uint32_t attack_plan_hold(uint32_t plan) {  // AI:255-312
  return plan == AP_ONE_HIT || plan == AP_TWO_HIT ? 1u : plan == AP_IMMEDIATE_SPECIAL ? 60u
       : plan == AP_DELAY_SPECIAL ? 120u : 0u;
}

// The plan choices as (n, outcome of Random.Range(0, n) = r) per distance bucket
// b = [d > 4, d > 3, d > 2.5, d > 2, else] (SelectMovement AI:68-126, SelectAttack AI:128-190).
constexpr uint32_t move_draw_n(int b) { return b == 0 ? 2u : b == 1 ? 7u : b == 2 ? 5u : b == 3 ? 4u : 3u; }
constexpr uint32_t move_draw_plan(int b, uint32_t r) {
  switch (b) {
    case 0: return r == 0 ? MP_FAR1 : MP_FAR2;
    case 1: return r <= 1 ? MP_MID1 : r <= 3 ? MP_MID2 : r == 4 ? MP_FAR1 : r == 5 ? MP_FAR2 : MP_NEUTRAL;
    case 2: return r == 0 ? MP_MID1 : r == 1 ? MP_MID2 : r == 2 ? MP_FALLBACK1 : r == 3 ? MP_FALLBACK2 : MP_NEUTRAL;
    case 3: return r == 0 ? MP_FALLBACK1 : r == 1 ? MP_FALLBACK2 : MP_NEUTRAL;
    default: return r == 0 ? MP_FALLBACK1 : r == 1 ? MP_FALLBACK2 : MP_NEUTRAL;
  }
}
constexpr uint32_t attack_draw_n(int b) { return b == 0 ? 4u : b == 1 ? 5u : b == 2 ? 3u : b == 3 ? 6u : 3u; }
constexpr uint32_t attack_draw_plan(int b, uint32_t r) {
  switch (b) {
    case 0: return r <= 3 ? AP_NONE : AP_DELAY_SPECIAL;
    case 1: return r <= 1 ? AP_NONE : r <= 3 ? AP_ONE_HIT : AP_DELAY_SPECIAL;
    case 2: return r == 0 ? AP_NONE : r == 1 ? AP_ONE_HIT : AP_TWO_HIT;
    case 3: return r <= 1 ? AP_ONE_HIT : r <= 3 ? AP_TWO_HIT : r == 4 ? AP_IMMEDIATE_SPECIAL : AP_DELAY_SPECIAL;
    default: return r == 0 ? AP_ONE_HIT : AP_TWO_HIT;
  }
}
// SelectAttack's answers that take no Random.Range draw: a hit/special/guard-break opponent
// (any distance), or an attacking one at 3 < d <= 4
__device__ __forceinline__ bool attack_forced(uint32_t b, uint32_t opp) {
  constexpr uint32_t kAny = (1u << A_DAMAGE) | (1u << A_GUARD_BREAK) | (1u << A_N_SPECIAL) | (1u << A_B_SPECIAL);
  constexpr uint32_t kMid = (1u << A_N_ATTACK) | (1u << A_B_ATTACK);
  return (((b == 1 ? kAny | kMid : kAny) >> opp) & 1u) != 0;
}

// The bot as tables (staged into LDS with the frame data), per queue q (0 = attack, 1 =
// movement): plan inputs as 2-bit codes (movement: Left / Right bits; attack: 1 = Attack
// pressed), one draw descriptor per distance bucket, plan lengths.
struct alignas(16) BotDraw {
  uint32_t map;    // nibble r = the plan drawn for r
  uint32_t magic;  // ceil(2^23 / n) (< 2^23): floor(v n^-1) = (v magic) >> 23 for v < 2^20, n < 8
  uint32_t n;
  uint32_t c16;    // 65536 % n
};
struct alignas(16) BotTables {
  BotDraw draw[2][5];       // [queue][bucket]
  uint32_t codes[2][8][8];  // [queue][plan][i >> 4]: the input of index i at bits 2 (i & 15)
  uint8_t len[2][8];        // [queue][plan]
};
constexpr BotDraw make_draw(uint32_t n, uint32_t map) {
  return BotDraw{map, (uint32_t)(((1u << 23) + n - 1) / n), n, 65536u % n};
}
constexpr BotTables make_bot_tables() {
  BotTables t{};
  for (int b = 0; b < 5; b++) {
    uint32_t mm = 0, ma = 0;
    for (uint32_t r = 0; r < move_draw_n(b); r++) mm |= move_draw_plan(b, r) << (4 * r);
    for (uint32_t r = 0; r < attack_draw_n(b); r++) ma |= attack_draw_plan(b, r) << (4 * r);
    t.draw[1][b] = make_draw(move_draw_n(b), mm);
    t.draw[0][b] = make_draw(attack_draw_n(b), ma);
  }
  for (uint32_t p = 0; p < 7; p++) {
    t.len[1][p] = (uint8_t)move_plan_len(p);
    for (uint32_t i = 0; i < move_plan_len(p); i++) t.codes[1][p][i >> 4] |= move_plan_input(p, i) << (2 * (i & 15));
  }
  for (uint32_t p = 0; p < 5; p++) {  // Attack held for the first frames; AP_TWO_HIT presses again at index 4
    t.len[0][p] = (uint8_t)attack_plan_len(p);
    for (uint32_t i = 0; i < attack_plan_len(p); i++)
      t.codes[0][p][i >> 4] |= (uint32_t)((i < attack_plan_hold(p)) | ((p == AP_TWO_HIT) & (i == 4))) << (2 * (i & 15));
  }
  return t;
}
static_assert(move_plan_len(MP_FAR1) <= 8 * 16 && attack_plan_len(AP_DELAY_SPECIAL) <= 8 * 16,
              "plans fit eight code words");
__constant__ const BotTables kBot = make_bot_tables();
__shared__ BotTables sBot;
template <bool G>
__device__ __forceinline__ const BotTables& bots() {
  if constexpr (G) return kBot;
  else return sBot;
}

// Copy the kTables image (fs_tables.h) and, for kernels with a scripted bot (BOTS), the bot
// tables into LDS by LDS-DMA (global_load_lds_dwordx4: L2 -> LDS with no VGPR round trip, 1 KB
// per wave instruction, 8 per wave for the 31 KB image).  The DMA lands at a wave-uniform LDS
// base + lane x 16, so each wave instruction fills one contiguous 1 KB piece of the image.
// All threads of the block must call this before any early return.
typedef __attribute__((address_space(1))) void* GlobalPtr;
typedef __attribute__((address_space(3))) void* LdsPtr;
template <int BYTES>
__device__ __forceinline__ void lds_dma_copy(void* dst, const void* src) {
  static_assert(BYTES % 16 == 0, "16-byte pieces");
  constexpr int kChunks = BYTES / 16, kPieces = (kChunks + 63) / 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int j = wave; j < kPieces; j += kBlock / 64) {  // wave-uniform
    const int c = j * 64 + lane;
    if (c < kChunks)
      __builtin_amdgcn_global_load_lds((GlobalPtr)(reinterpret_cast<const char*>(src) + c * 16),
                                       (LdsPtr)(reinterpret_cast<char*>(dst) + j * 1024), 16, 0, 0);
  }
}
template <bool BOTS = true>
__device__ __forceinline__ void stage_tables() {
  lds_dma_copy<sizeof(Tables)>(&sT, &kTables);
  if constexpr (BOTS) lds_dma_copy<sizeof(BotTables)>(&sBot, &kBot);
  __syncthreads();  // (waits for the DMA: it counts on vmcnt)
}

// Random.Range(0, n) = x % n for the draw descriptor: x = h 2^16 + l, so x % n = (h (2^16 % n) + l) % n
// with the inner value v < 2^19.  The quotient is (v magic) >> 23 with magic = ceil(2^23 / n): the
// product exceeds v / n by less than v / 2^23 < 1/8 < 1/n, which cannot carry past the next
// integer.  Every factor is below 2^24, so the product is two full-rate 24-bit multiplies
// (v_mul_u32_u24 / v_mul_hi_u32_u24, bits 31:0 and 47:32) instead of the quarter-rate 32-bit ones.
__device__ __forceinline__ uint32_t draw_mod(uint32_t x, const BotDraw& d) {
  const uint32_t v = __umul24(x >> 16, d.c16) + (x & 0xFFFFu);
  const uint64_t prod = (uint64_t)(v & 0xFFFFFFu) * (uint64_t)(d.magic & 0xFFFFFFu);  // 24 x 24 bits
  const uint32_t q = (uint32_t)(prod >> 23);
  return v - __umul24(d.n, q);
}

// getNextAIInput (AI:41-66) for the P2 bot.  The ascending copy loop of
// UpdateFightState (AI:358-361) leaves fightStates[5] == the *previous* call's
// state, so the bot keeps one FightState: (distance, opponent action).
// The two lanes of an arena share the bot: each runs one of its two input queues (the P1 lane
// the attack queue, the P2 lane the movement queue) and both keep replicas of the RNG and of
// the previous FightState, so one pass of the same instructions serves both queues.
struct Bot {
  uint4 rng;               // replica on both lanes
  uint32_t plan, idx;      // this lane's queue: plan stored + 1 (0 = empty), index into it
  uint32_t prev_opp;       // replica
  float prev_dist;         // replica
};

// Mathf.Abs(fighter2.x - fighter1.x) (AI:370-373)
template <int FM>
__device__ __forceinline__ float bot_distance(float x1, float x2) {
  return fabsf(fsub<FM>(x2, x1));
}

// Branch-free over the pair: this lane's queue input from the code tables, both queues' busy
// flags (one exchange), both possible draws for the RNG (movement first, then attack -- the order
// the C# calls Random.Range), this queue's draw, and the RNG advanced by the number taken.
// q = this lane's queue (0 = attack on the P1 lane, 1 = movement on the P2 lane).  Both lanes of
// the pair must call it (it exchanges with the partner); it returns the bot's input on both.
__device__ __forceinline__ uint32_t xpair(uint32_t v);
// The bot tables one call reads depend only on the bot's state before the call (its queue's plan
// and index, the previous FightState's distance bucket), so the fused tick issues them at its
// start (bot_prefetch) and the call at its end finds them resident.
struct BotPre {
  uint32_t code_word;  // codes[q][plan][idx >> 4]
  BotDraw w;           // draw[q][bucket of the previous distance]
  uint32_t len;        // len[q][plan]
};
__device__ __forceinline__ uint32_t bot_bucket(float d) {
  return d > 4.0f ? 0u : d > 3.0f ? 1u : d > 2.5f ? 2u : d > 2.0f ? 3u : 4u;
}
template <bool G>
__device__ __forceinline__ BotPre bot_prefetch(const Bot& b, uint32_t q) {
  const uint32_t p = b.plan != 0 ? b.plan - 1 : 0u;
  BotPre r;
  r.code_word = bots<G>().codes[q][p][b.idx >> 4];
  r.w = bots<G>().draw[q][bot_bucket(b.prev_dist)];
  r.len = bots<G>().len[q][p];
  return r;
}

template <bool G>
__device__ __forceinline__ uint32_t bot_next_input(Bot& b, uint32_t q, float dist, uint32_t opp_act, const BotPre& pre) {
  const float d = b.prev_dist;
  const uint32_t opp = b.prev_opp;
  b.prev_dist = dist;
  b.prev_opp = opp_act;
  const uint32_t bucket = bot_bucket(d);
  const bool busy = b.plan != 0;
  const uint32_t i = b.idx;  // (the plan's code word and length came with the prefetch)
  const uint32_t code = (pre.code_word >> (2 * (i & 15))) & 3u;
  const uint32_t mine = busy ? (q ? code : code << 2) : 0u;  // Left / Right bits, or IN_ATTACK
  const bool o_busy = xpair((uint32_t)busy) != 0;
  const bool mbusy = q ? busy : o_busy, abusy = q ? o_busy : busy;
  const bool forced = attack_forced(bucket, opp);
  const bool dm = !mbusy, da = !abusy & !forced;
  uint4 s1 = b.rng;
  const uint32_t x1 = rng_next(s1);
  uint4 s2 = s1;
  const uint32_t x2 = rng_next(s2);
  const uint4 s0 = b.rng;
  b.rng = sel4(dm & da, s2, sel4(dm | da, s1, s0));
  const BotDraw w = pre.w;
  const uint32_t drawn = (w.map >> (4 * draw_mod((!q & dm) ? x2 : x1, w))) & 15u;
  const uint32_t newp = (!q & forced) ? (uint32_t)AP_TWO_HIT : drawn;
  const uint32_t i1 = i + 1;
  b.plan = busy ? (i1 == pre.len ? 0u : b.plan) : newp + 1;
  b.idx = busy ? i1 : 0u;
  return mine | xpair(mine);
}

// The whole BattleAI of one fighter on one lane (both queues), for the per-arena actor variant
// (kActors): P1's bot (by_example) on the P1 lane, P2's on the P2 lane, the game's one RNG passed
// between them in TrainingManager.Step's order (P1 first).  Off the throughput path, so written
// with plain branches.
struct FullBot {
  uint32_t mplan, midx, aplan, aidx;  // plans stored + 1 (0 = empty queue)
  uint32_t prev_opp;                  // fightStates[5]: opponent action idx ...
  float prev_dist;                    // ... and distance
  bool ready;                         // fightStates[5] != null
};

__device__ __forceinline__ FullBot unpack_bot(uint2 w, uint32_t& input) {
  FullBot b;
  b.mplan = w.x & 7;
  b.midx = (w.x >> 3) & 127;
  b.aplan = (w.x >> 10) & 7;
  b.aidx = (w.x >> 13) & 127;
  b.prev_opp = (w.x >> 20) & 31;
  b.ready = (w.x >> 25) & 1;
  input = (w.x >> 26) & 7;
  b.prev_dist = __uint_as_float(w.y);
  return b;
}
__device__ __forceinline__ uint2 pack_bot(const FullBot& b, uint32_t input) {
  return make_uint2(b.mplan | (b.midx << 3) | (b.aplan << 10) | (b.aidx << 13) | (b.prev_opp << 20) |
                        ((uint32_t)b.ready << 25) | (input << 26),
                    __float_as_uint(b.prev_dist));
}

// getNextAIInput (AI:41-66) of fighter k's bot: UpdateFightState (AI:344-363) first, then the
// previous call's state decides; a bot whose fightStates[5] is still null (never Reset, first
// call) answers 0 without touching its queues or the RNG.  P1's forward is Right (AI:380-388),
// so its movement codes are mirrored.
template <bool G>
__device__ __forceinline__ uint32_t bot_full_next(FullBot& b, uint4& rng, uint32_t k, float dist, uint32_t opp_act) {
  const bool ready = b.ready;
  const float d = b.prev_dist;
  const uint32_t opp = b.prev_opp;
  b.prev_dist = dist;
  b.prev_opp = opp_act;
  b.ready = true;
  if (!ready) return 0u;
  const uint32_t bucket = d > 4.0f ? 0u : d > 3.0f ? 1u : d > 2.5f ? 2u : d > 2.0f ? 3u : 4u;
  uint32_t in = 0;
  if (b.mplan != 0) {  // moveQueue.Dequeue
    const uint32_t p = b.mplan - 1, i = b.midx;
    const uint32_t c = (bots<G>().codes[1][p][i >> 4] >> (2 * (i & 15))) & 3u;
    in |= k == 0 ? (((c & 1u) << 1) | (c >> 1)) : c;
    b.midx = i + 1;
    if (b.midx == bots<G>().len[1][p]) b.mplan = 0;
  } else {  // SelectMovement (AI:68-126)
    const BotDraw w = bots<G>().draw[1][bucket];
    b.mplan = ((w.map >> (4 * draw_mod(rng_next(rng), w))) & 15u) + 1;
    b.midx = 0;
  }
  if (b.aplan != 0) {  // attackQueue.Dequeue
    const uint32_t p = b.aplan - 1, i = b.aidx;
    in |= ((bots<G>().codes[0][p][i >> 4] >> (2 * (i & 15))) & 1u) << 2;
    b.aidx = i + 1;
    if (b.aidx == bots<G>().len[0][p]) b.aplan = 0;
  } else if (attack_forced(bucket, opp)) {  // SelectAttack without a draw (AI:130-133, 147-151)
    b.aplan = AP_TWO_HIT + 1;
    b.aidx = 0;
  } else {  // SelectAttack (AI:128-190)
    const BotDraw w = bots<G>().draw[0][bucket];
    b.aplan = ((w.map >> (4 * draw_mod(rng_next(rng), w))) & 15u) + 1;
    b.aidx = 0;
  }
  return in;
}

// BattleAI.Reset (AI:393-403): empty queues, every FightState slot = the current state
__device__ __forceinline__ void bot_full_reset(FullBot& b, float dist, uint32_t opp_act) {
  b.mplan = b.midx = b.aplan = b.aidx = 0;
  b.prev_dist = dist;
  b.prev_opp = opp_act;
  b.ready = true;
}

// ---------------------------------------------------------------------------
// Two lanes per arena.  Lane 2a+k runs fighter k of arena a (k = 0: P1, faces
// right; k = 1: P2).  Per-fighter phases (UpdateInput .. UpdateBoxes) run on
// both lanes at once; the pair phases (character push, hit/hurt collision, KO,
// reward) exchange the partner's values with one DPP quad_perm [1,0,3,2] move
// per 32-bit value.  Arena-level fields (frameCount, recording count, reward
// accumulator, reset flags) are kept as identical replicas on both lanes and
// stored by lane k = 0; the bot's two queues are split over the pair.  Every exchange sits in
// control flow that is uniform across a pair, so the partner lane is active.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xpair(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1 /* quad_perm(1,0,3,2) */, 0xF, 0xF, true);
}
__device__ __forceinline__ int xpair(int v) { return (int)xpair((uint32_t)v); }
__device__ __forceinline__ float xpair(float v) { return __uint_as_float(xpair(__float_as_uint(v))); }
// P1's / P2's value of the pair on both lanes (quad_perm [0,0,2,2] / [1,1,3,3]): one DPP move
// instead of an exchange plus a lane-parity select
__device__ __forceinline__ uint32_t xp1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0 /* quad_perm(0,0,2,2) */, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t xp2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5 /* quad_perm(1,1,3,3) */, 0xF, 0xF, true);
}
__device__ __forceinline__ float xp1(float v) { return __uint_as_float(xp1(__float_as_uint(v))); }
__device__ __forceinline__ float xp2(float v) { return __uint_as_float(xp2(__float_as_uint(v))); }

struct Lane {
  Fighter f;
  uint32_t k;         // 0: P1, 1: P2
  int frame_count;    // replicas ...
  uint32_t rec_count;
  uint32_t pending, has_term;  // 0 / 1
  double cum;
  uint32_t rec;       // this player's recordingPnInput[index - 1]
  uint32_t act;       // this player's remote actor's input (TrainingRemoteActor.input)
  uint32_t bin;       // this player's bot actor's input (TrainingBattleAIActor.input), bot lanes only
  uint32_t p2bot;     // kActors: P2's actor is the bot (replica)
  AInfo ai;           // ActionInfo of f.act (reloaded at the end of every tick)
  Bot bot;            // FS_P2_BOT only: this lane's queue + replicas (see Bot)
  FullBot fb;         // kActors only: this fighter's whole BattleAI
  uint4 rng;          // kActors only: the game's RNG (replica)
};

template <int V>
__device__ __forceinline__ void load_lane(Lane& L, const DevState& s, int a, uint32_t k) {
  const int l = 2 * a + (int)k;
  L.k = k;
  L.f.x = reinterpret_cast<const float*>(s.pos)[l];
  L.f.hist = reinterpret_cast<const uint32_t*>(s.hist)[l];
  const uint2 w = reinterpret_cast<const uint2*>(s.fpk)[l];
  const int2 aw = s.aw[a];
  L.cum = s.cum[a];
  unpack_fighter(L.f, w.x, w.y);
  const uint32_t h = (uint32_t)aw.y;
  L.frame_count = aw.x;
  L.rec_count = h & 0x7fff;
  L.rec = (h >> (k ? 18 : 15)) & 7;
  L.act = (h >> (k ? 24 : 21)) & 7;
  L.pending = (h >> 27) & 1;
  L.has_term = (h >> 28) & 1;
  L.p2bot = (h >> 29) & 1;
  L.bin = 0;
  if constexpr (V == FS_P2_BOT) {  // both lanes read the same 24 B (one cache line); P2 uses it
    L.bot.rng = s.rng[a];
    const uint2 b = s.bot[a];
    L.bot.plan = k ? (b.x & 7) : ((b.x >> 10) & 7);  // P2 lane: movement queue, P1 lane: attack queue
    L.bot.idx = k ? ((b.x >> 3) & 127) : ((b.x >> 13) & 127);
    L.bot.prev_opp = (b.x >> 20) & 31;
    L.bot.prev_dist = __uint_as_float(b.y);
    L.bin = (b.x >> 26) & 7;  // (a bot-created P2 is Reset at every Intro: always ready)
  } else if constexpr (V == kActors) {
    L.rng = s.rng[a];
    L.fb = unpack_bot(k ? s.bot[a] : s.bot1[a], L.bin);
  }
}

template <int V>
__device__ __forceinline__ void store_lane(const Lane& L, const DevState& s, int a) {
  const int l = 2 * a + (int)L.k;
  const uint64_t w = pack_fighter(L.f);
  reinterpret_cast<float*>(s.pos)[l] = L.f.x;
  reinterpret_cast<uint32_t*>(s.hist)[l] = L.f.hist;
  reinterpret_cast<uint2*>(s.fpk)[l] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
  const uint32_t other = xpair(L.rec | (L.act << 3));  // P2's recorded/actor input for the header
  if (L.k == 0) {
    const uint32_t p2bot = V == FS_P2_BOT ? 1u : V == kActors ? (uint32_t)L.p2bot : 0u;
    const uint32_t h = L.rec_count | (L.rec << 15) | ((other & 7) << 18) | (L.act << 21) | ((other >> 3) << 24) |
                       ((uint32_t)L.pending << 27) | ((uint32_t)L.has_term << 28) | (p2bot << 29);
    s.aw[a] = make_int2(L.frame_count, (int)h);
    s.cum[a] = L.cum;
  }
  if constexpr (V == FS_P2_BOT) {
    const Bot& b = L.bot;
    const uint32_t mine = b.plan | (b.idx << 3), other = xpair(mine);  // the partner's queue
    if (L.k == 1) {
      s.rng[a] = b.rng;
      s.bot[a] = make_uint2(mine | (other << 10) | (b.prev_opp << 20) | (1u << 25) | (L.bin << 26),
                            __float_as_uint(b.prev_dist));
    }
  } else if constexpr (V == kActors) {
    const uint2 bw = pack_bot(L.fb, L.bin);
    if (L.k == 1) {
      s.rng[a] = L.rng;
      s.bot[a] = bw;
    } else {
      s.bot1[a] = bw;
    }
  }
}

// UpdatePushCharacterVsCharacter (BC:483-501) with UnityEngine.Rect semantics:
// x is xMin, xMax = width + x, Overlaps is strict; each lane applies its own fighter's
// shift.  The y-test is constant: tools/gen_tables.py proves every pair of pushboxes
// overlaps vertically (kPushYAlwaysOverlaps) and keeps no y extents in the records.
static_assert(kPushYAlwaysOverlaps, "the frame records keep no pushbox y extents");
template <int FM, bool GEOM = false>
__device__ __forceinline__ void push_character_vs_character(Fighter& f, uint32_t k, float ph = 0.0f) {
  // The test and the shift are symmetric in the two fighters, so each lane evaluates them
  // as (mine, partner's) -- the same operations on the same values as (P1, P2).
  const float o_px = xpair(f.px), o_x = xpair(f.x), o_pw = xpair(f.pw);
  const float xmax_m = fadd<FM>(f.pw, f.px), xmax_o = fadd<FM>(o_pw, o_px);  // Rect.xMax = width + x
  bool overlap = (xmax_o > f.px) & (o_px < xmax_m);
  float o_y = 0.0f;
  if constexpr (GEOM) {  // the y half of Rect.Overlaps (yMax = height + y), ph = my pushbox height
    const float o_py = xpair(f.py), o_ph = xpair(ph);
    o_y = xpair(f.y);
    const float ymax_m = fadd<FM>(ph, f.py), ymax_o = fadd<FM>(o_ph, o_py);
    overlap = overlap & (ymax_o > f.py) & (o_py < ymax_m);
  }
  if (!overlap || f.x == o_x) return;  // a tie pushes nothing (BC:490-499)
  const bool left = f.x < o_x;         // the left fighter moves by -d/2, the right one by +d/2
  float dx;
  if constexpr (FM == FS_FLOAT_DOUBLE) {
    const double d = left ? (double)xmax_m - (double)o_px : (double)xmax_o - (double)f.px;
    dx = left ? (float)(d * -1 / 2) : (float)(d * 1 / 2);
  } else {
    const float d = left ? __fsub_rn(xmax_m, o_px) : __fsub_rn(xmax_o, f.px);
    dx = left ? d * -1.0f / 2.0f : d * 1.0f / 2.0f;
  }
  apply_position_change<FM>(f, dx);
  // P1 shifts by its own y; P2 by its own when P1 is on the left, else by P1's y after P1's shift
  if constexpr (GEOM) apply_position_change_y<FM>(f, (k == 1 && o_x > f.x) ? fadd<FM>(o_y, o_y) : f.y);
}

// UpdateHitboxHurtboxCollision (BC:521-591): attacker P1 (phase A), then attacker P2
// (phase B).  The boxes are those of UpdateBoxes (not rebuilt when a hit changes an
// action), but phase B re-reads P2's hit count, which phase A resets if it hit P2
// (sequential trade semantics).  Each lane tests the partner's hitboxes against its
// own hurtboxes in one pass -- the P2 lane is phase A's defender, the P1 lane phase
// B's -- and phase B is resolved for both possible P2 hit counts, so only the
// outcomes cross the pair: A's result to P1 (NotifyAttackHit), whether P2 was hit to
// P1 (to pick B's variant), B's result to P2, and each defender's stun to the other.
// The record boxes (my hurtboxes, the partner's hitboxes) are read from LDS together with
// the frame record (one round trip) rather than here.
__device__ __forceinline__ uint32_t bit0_mask(uint32_t v) { return (uint32_t)((int32_t)(v << 31) >> 31); }  // 0 / ~0

// AttackData of attack index i (kAttacks, fs_tables.h) selected in registers: the hit path
// makes no LDS round trip for it.
constexpr uint32_t attack_word(int j, int w) {
  return w == 0 ? (uint32_t)kAttacks[j].damage_action | ((uint32_t)kAttacks[j].guard_action << 8) |
                      ((uint32_t)kAttacks[j].number_of_hit << 16) | ((uint32_t)kAttacks[j].vital_damage << 24)
                : (uint32_t)kAttacks[j].guard_damage | ((uint32_t)kAttacks[j].hit_stun << 8) |
                      ((uint32_t)kAttacks[j].guard_stun << 16) | ((uint32_t)kAttacks[j].guard_break_stun << 24);
}
template <int W>
__device__ __forceinline__ uint32_t attack_word_sel(bool b1, bool b2) {
  constexpr uint32_t a0 = attack_word(0, W), a1 = attack_word(1, W), a2 = attack_word(2, W), a3 = attack_word(3, W);
  return b2 ? (b1 ? a3 : a2) : (b1 ? a1 : a0);
}
__device__ __forceinline__ AttackInfo attack_info(int i) {
  static_assert(sizeof(AttackInfo) == 8, "AttackInfo is two words");
  static_assert(sizeof(kAttacks) / sizeof(kAttacks[0]) == 4, "four attacks");
  const bool b1 = i & 1, b2 = i & 2;
  const uint32_t w[2] = {attack_word_sel<0>(b1, b2), attack_word_sel<1>(b1, b2)};
  AttackInfo a;
  a.damage_action = (uint8_t)w[0];
  a.guard_action = (uint8_t)(w[0] >> 8);
  a.number_of_hit = (uint8_t)(w[0] >> 16);
  a.vital_damage = (uint8_t)(w[0] >> 24);
  a.guard_damage = (uint8_t)w[1];
  a.hit_stun = (uint8_t)(w[1] >> 8);
  a.guard_stun = (uint8_t)(w[1] >> 16);
  a.guard_break_stun = (uint8_t)(w[1] >> 24);
  return a;
}

// `res` = kTables.resolve[o_hits * kNumFrameRecs + o_rec], read with the frame record: byte m (the box-pair
// overlap mask) holds the outcome at the attacker's hit count o_hits (low nibble) and at 0 (high).
template <int FM>
__device__ __forceinline__ void hitbox_hurtbox_collision(Fighter& f, uint32_t k, F4 my_hurt, float o_hw0, float o_hw1,
                                                         U4 res, uint32_t ym) {
  // (no wave-level skip: absent hitboxes never overlap in y, ybits)
  const float o_hx0 = xpair(f.hx0), o_hx1 = xpair(f.hx1);
  const uint32_t xm = box_x_overlaps<FM>(o_hw0, o_hw1, o_hx0, o_hx1, my_hurt.zw, F2{f.ux0, f.ux1});
  // phase A (P1 attacks P2) is resolved on the P2 lane; its outcome crosses to P1, whose lane
  // then resolves phase B (P2 attacks P1) with P2's hit count after phase A
  // the resolution for both phases from one byte of the attacker's entry (kTables.resolve,
  // tools/gen_tables.py), picked by v_perm_b32 (selector byte m & 7 of the low or high 8 bytes;
  // selector 0x0c = zero)
  const uint32_t m = xm & ym;
  const uint32_t sel = (m & 7u) | 0x0c0c0c00u;
  const uint32_t lo = __builtin_amdgcn_perm(res.y, res.x, sel), hi = __builtin_amdgcn_perm(res.w, res.z, sel);
  const uint32_t tab = (m & 8u) ? hi : lo;
  // On the P2 lane phase A's outcome (at P1's hit count); on the P1 lane phase B's, unless phase
  // A hit P2 -- which resets P2's hit count to 0 first (SetCurrentAction), so P1 then reads the
  // outcome at hit count 0.
  // (every exchange is its own statement on both lanes: inside a select the compiler may run
  // the DPP move under a one-lane exec mask, and a disabled source lane reads as 0)
  const uint32_t t1 = tab & 15u;
  const uint32_t hitA = xp2(t1) & 1u;  // phase A's outcome, from the P2 lane
  const uint32_t t = (k == 0 && hitA) ? (tab >> 4) : t1;  // this lane's phase as the defender
  const bool my_hit = (t & 1u) != 0;
  const int my_atk = (int)((t >> 1) & 3u);
  const bool my_prox = ((t >> 3) & 1u) != 0;
  // each lane is the defender of exactly one phase: one NotifyDamaged per lane.  Order per
  // fighter as in the reference: P1 gets NotifyAttackHit (A) before its NotifyDamaged (B);
  // P2 its NotifyDamaged (A) before NotifyAttackHit (B).
  f.hits += k == 0 ? (int)hitA : 0;  // NotifyAttackHit for P1 (F:352-355)
  int my_stun = 0;
  if (my_hit) {
    const AttackInfo ad = attack_info(my_atk);
    const int res = notify_damaged(f, ad);
    my_stun = res == DR_GUARD ? ad.guard_stun : res == DR_GUARD_BREAK ? ad.guard_break_stun : ad.hit_stun;
  }
  if (!my_hit && my_prox && f.in_back) f.prox = true;  // NotifyInProximityGuardRange (F:400-406)
  // (hit, stun) of both defenders: pA = P2's (phase A), pB = P1's (phase B)
  const uint32_t mine = (uint32_t)my_hit | ((uint32_t)my_stun << 1);
  const uint32_t pA = xp2(mine), pB = xp1(mine);
  f.hits += k == 1 ? (int)(pB & 1u) : 0;  // NotifyAttackHit for P2
  // SetHitStun on both, phase B last (BC:576-578), as bit-mask selects (v_bfe_i32 + v_bfi_b32:
  // written as ?: the compiler branches here)
  const uint32_t mA = bit0_mask(pA), mB = bit0_mask(pB);
  const uint32_t sA = (mA & (pA >> 1)) | (~mA & (uint32_t)f.stun);
  f.stun = (int)((mB & (pB >> 1)) | (~mB & sA));
}

// KO tick -> End (winner), End tick (BC:221-243, 306-325, 371-381), reduced to
// its observable effects.  SetupBattleStart (next tick) overwrites position,
// action, frame, hit count, buffer, reserve, vital, guard, hasWon and the input
// history, so what survives the End tick is (a) the hitstun decrement and (b)
// UpdateActionRequest clearing isInputBackward / isReserveProximityGuard --
// unless it returned early: for the winner (hasWon), or on the reserve / buffer
// paths (F:204-229).  The history was cleared at KO, so the fall-through sees no input.
__device__ __forceinline__ void end_tick(Fighter& f, bool won) {
  f.stun -= f.stun > 0 ? 1 : 0;
  const bool early = won || (f.rsv != NONE && f.stun <= 0) ||
                     (f.buf != NONE && (kCanCancelOnWhiff || f.hits > 0) && f.stun <= 0);
  f.in_back = early ? f.in_back : false;
  f.prox = early ? f.prox : false;
}

// SetupBattleStart (F:120-135): hitstun and the two guard latches are NOT reset
// (position.y = 0 and isFaceRight = isPlayerOne, F:123-124, BC:264-265, are set by the callers
// that carry them: the general-geometry tick and the reset kernel; on the standard tick both
// already hold.)
__device__ __forceinline__ void setup_battle_start(Fighter& f, float x) {
  f.x = x;
  f.vital = 1;
  f.guard = kStartGuard;
  f.won = false;
  f.hist = 0;
  f.hold = 0;
  set_action(f, A_STAND);
}

// The reset burst of one lane (BC:212-345).  after_ko: the KO -> End -> Stop ->
// Intro -> Fight sequence after a terminal frame (ClearInput already applied);
// otherwise the RESET / game-start path Stop -> Intro -> Fight.
//   Intro tick: the stale actor input enters the cleared history, the frame
//   advances unless in hitstun, RequestAction(STAND) on STAND is a no-op, and
//   movement / boxes / pushes are no-ops (STAND has no movement window; base
//   pushboxes at x = -2 / +2 neither overlap nor touch the stage edges).
//   Fight: frameCount = -1, recording index 0, state(-1) emitted, and the bot's
//   first RequestNextInput.
// The handle's actors, for kActors (StepParams / ResetParams).
struct Actors {
  bool p1_bot;     // FS_P1_BOT
  bool p2_resets;  // P2's bot is Reset at Intro (a bot-created P2)
  bool p2_noop;    // a non-bot P2 presses nothing
};

// The actor input this lane's fighter gets this frame when no new action arrives (Intro, and
// every frame for a bot): TrainingActor.GetInput() of the player's current actor.
template <int V>
__device__ __forceinline__ uint32_t stored_input(const Lane& L, const Actors& ac) {
  if constexpr (V == FS_P2_BOT) return L.k == 1 ? L.bin : L.act;
  else if constexpr (V == kActors)
    return (L.k == 0 ? ac.p1_bot : L.p2bot) ? L.bin : ((L.k == 1 && ac.p2_noop) ? 0u : L.act);
  else if constexpr (V == FS_P2_NOOP) return L.k == 1 ? 0u : L.act;  // an idle P2 presses nothing
  else return L.act;
}

// TrainingManager.Step's RequestNextInput for kActors: P1's bot, then P2's (TrainingManager.cs:
// 59-77), each on its own lane, the RNG handed from one to the other.  Both lanes must call it.
__device__ __forceinline__ uint4 xpair4(uint4 v) {
  uint4 o;
  o.x = xpair(v.x);
  o.y = xpair(v.y);
  o.z = xpair(v.z);
  o.w = xpair(v.w);
  return o;
}
template <bool G>
__device__ __forceinline__ void actors_request(Lane& L, const Actors& ac, float dist, uint32_t p1_act,
                                               uint32_t p2_act) {
  uint4 r = L.rng;
  if (ac.p1_bot) {
    if (L.k == 0) L.bin = bot_full_next<G>(L.fb, r, 0, dist, p2_act);
    const uint4 o = xpair4(r);
    r = sel4(L.k == 1, o, r);
  }
  if (L.p2bot) {
    if (L.k == 1) L.bin = bot_full_next<G>(L.fb, r, 1, dist, p1_act);
    const uint4 o = xpair4(r);
    r = sel4(L.k == 0, o, r);
  }
  L.rng = r;
}

// The reset burst of one lane (BC:212-345).  after_ko: the KO -> End -> Stop ->
// Intro -> Fight sequence after a terminal frame (ClearInput already applied);
// otherwise the RESET / game-start path Stop -> Intro -> Fight.
//   Intro: SetupBattleStart, then the bots' Reset -- P2's only when it is the bot the game was
//   launched with (--p2-bot); a bot switched in by P2_BOT is never Reset (BC:276-277 throws on the
//   null GameManager.botP2 first) and P1's spectator-wrapped bot is not a TrainingBattleAIActor.
//   Intro tick: the stale actor input enters the cleared history, the frame
//   advances unless in hitstun, RequestAction(STAND) on STAND is a no-op, and
//   movement / boxes / pushes are no-ops (STAND has no movement window; base
//   pushboxes at x = -2 / +2 neither overlap nor touch the stage edges).
//   Fight: frameCount = -1, recording index 0, state(-1) emitted, and the bots'
//   first RequestNextInput.
template <int FM, int V, bool G = false>
__device__ __forceinline__ void reset_burst(Lane& L, bool after_ko, const Actors& ac) {
  constexpr bool BOT = V == FS_P2_BOT;
  if (after_ko) {
    const int o_vital = xpair(L.f.vital);
    end_tick(L.f, L.f.won || (L.f.vital > 0 && o_vital <= 0));  // a sole survivor wins (BC:310-323)
  }
  setup_battle_start(L.f, L.k == 0 ? kP1StartX : kP2StartX);
  const float o_x = xpair(L.f.x);
  const uint32_t o_act = xpair((uint32_t)L.f.act);
  const float x1 = L.k == 0 ? L.f.x : o_x, x2 = L.k == 0 ? o_x : L.f.x;
  const uint32_t p1_act = L.k == 0 ? (uint32_t)L.f.act : o_act;
  const uint32_t p2_act = L.k == 1 ? (uint32_t)L.f.act : o_act;
  if constexpr (BOT) {  // BattleAI.Reset (AI:393-403)
    L.bot.plan = L.bot.idx = 0;
    L.bot.prev_dist = bot_distance<FM>(x1, x2);
    L.bot.prev_opp = p1_act;
  } else if constexpr (V == kActors) {
    if (L.k == 1 && L.p2bot && ac.p2_resets) bot_full_reset(L.fb, bot_distance<FM>(x1, x2), p1_act);
  }
  const uint32_t in = stored_input<V>(L, ac);
  if (L.rec_count < kMaxRecording) {  // RecordInput in the Intro tick (BC:333)
    L.rec = in;
    L.rec_count++;
  }
  const uint32_t r = rel_bits(in, (int)L.k);
  L.f.hist = (r & 1) | ((r & 2) << 15);
  L.f.hold = (in & IN_ATTACK) ? 1 : 0;
  const bool stunned = L.f.stun > 0;
  L.f.stun -= stunned ? 1 : 0;
  L.f.frame = stunned ? 0 : 1;
  L.frame_count = -1;
  L.rec_count = 0;
  if constexpr (BOT) {
    const uint32_t bi = bot_next_input<G>(L.bot, L.k, bot_distance<FM>(x1, x2), p1_act, bot_prefetch<G>(L.bot, L.k));
    L.bin = L.k == 1 ? bi : L.bin;
  } else if constexpr (V == kActors) {
    actors_request<G>(L, ac, bot_distance<FM>(x1, x2), p1_act, p2_act);
  }
}

// ---------------------------------------------------------------------------
// outputs (FE:336-380, 537-549): each lane writes its own column of the [N][2]
// pairs (one byte / float per lane, fully coalesced); lane k = 0 the per-arena ones
// ---------------------------------------------------------------------------
// Stores at a 32-bit byte offset from a kernel-argument base: the address is one SGPR pair plus
// one VGPR (global_store ... saddr), with no 64-bit address arithmetic per store.  The host
// splits launches so every trajectory offset fits (fs_api.cpp, kMaxLaunchRows).  The outputs
// stream out and are not read back by the launch, so the stores are non-temporal (`nt`): they
// do not pile up as dirty lines in L2 (1000-tick launches +4.8 %, 20-tick +2.4 %, A/B on one box).
template <class T>
__device__ __forceinline__ void st_off(T* base, uint32_t byte_off, T v) {
  __builtin_nontemporal_store(v, reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off));
}

__device__ __forceinline__ void write_obs(const Lane& L, uint8_t* guard, uint8_t* move, float* move_frame,
                                          float* position, int32_t* frame, uint8_t* action, uint8_t* hitstun,
                                          uint32_t r) {
  int a = L.f.act;
  if (a == A_DEAD || a == A_WIN) a = A_STAND;  // FE:537-549
  const int mf = (a == A_STAND || a == A_FORWARD || a == A_BACKWARD) ? 0 : L.f.frame;  // FE:339-358
  const uint32_t c = 2 * r + L.k;
  st_off(guard, c, (uint8_t)L.f.guard);
  st_off(move, c, (uint8_t)a);
  st_off(move_frame, 4 * c, (float)mf);
  st_off(position, 4 * c, L.f.x);
  st_off(action, c, L.rec_count > 0 ? (uint8_t)L.rec : (uint8_t)0);
  st_off(hitstun, c, (uint8_t)L.f.stun);
  st_off(frame, 4 * r, (int32_t)L.frame_count);  // both lanes hold the replica: the same value to the same address
}

__device__ __forceinline__ void write_main(const Lane& L, const DevOutputs& o, uint32_t r) {
  write_obs(L, o.guard, o.move, o.move_frame, o.position, o.frame, o.action, o.hitstun, r);
}
__device__ __forceinline__ void write_final(const Lane& L, const DevOutputs& o, uint32_t r) {
  write_obs(L, o.final_guard, o.final_move, o.final_move_frame, o.final_position, o.final_frame, o.final_action,
            o.final_hitstun, r);
}

// fs_step_n_packed (include/footsies.h fs_packed_traj): the values write_obs stores, as one 16-B
// record per lane -- the guard / move / action / hitstun bytes, move_frame, position and a fourth
// word w3 (P1: the frame; P2: the terminated / truncated bytes) -- so that a tick's outputs take
// two store instructions (this record and the f64 reward) instead of ten.
typedef uint32_t PkRec __attribute__((ext_vector_type(4)));  // a native vector: one 16-B store
__device__ __forceinline__ PkRec packed_record(const Lane& L, uint32_t w3) {
  int a = L.f.act;
  if (a == A_DEAD || a == A_WIN) a = A_STAND;  // FE:537-549
  const int mf = (a == A_STAND || a == A_FORWARD || a == A_BACKWARD) ? 0 : L.f.frame;  // FE:339-358
  const uint32_t act = L.rec_count > 0 ? (uint32_t)L.rec : 0u;  // a 3-bit input
  PkRec v;
  // (guard is 0..3, the move index 0..16, the input 0..7: each fits its byte as it is; the shift
  // keeps hitstun's low byte, the byte the per-field store keeps)
  v.x = (uint32_t)L.f.guard | ((uint32_t)a << 8) | (act << 16) | ((uint32_t)L.f.stun << 24);
  v.y = __float_as_uint((float)mf);
  v.z = __float_as_uint(L.f.x);
  v.w = w3;
  return v;
}
// lane record c = 2 r + k of row r (byte offset 16 c: the host keeps 32 r below 2^32)
__device__ __forceinline__ void write_packed(const Lane& L, uint4* base, uint32_t r, uint32_t w3) {
  st_off(reinterpret_cast<PkRec*>(base), 16u * (2u * r + L.k), packed_record(L, w3));
}

// fs_step_rec: arena r's FS_RECORD_BYTES gather record (fs_gather.hip k_pack_records' layout:
// guard[2] move[2] action[2] hitstun[2] terminated truncated pad[2] move_frame[2] position[2] frame
// reward) from the values write_obs stores.  Both lanes of the pair store 16 B in one instruction
// -- lane 0 bytes 0-15 (the byte fields, the flags, P1's move_frame), lane 1 bytes 16-31 (P2's
// move_frame, both positions, the frame) -- and lane 0 the f64 reward at byte 32: two stores per
// wave instead of five, after two pair exchanges.  Both lanes must call it (the exchanges read the
// partner's registers).  (The 16-B halves are 8-B aligned: 40 r + 16 k.)
typedef uint32_t RecQ __attribute__((ext_vector_type(4), aligned(8)));
__device__ __forceinline__ void write_record(const Lane& L, uint2* rec, uint32_t r, uint32_t terminated,
                                             double reward) {
  const PkRec v = packed_record(L, 0u);  // bytes guard | move | action | hitstun, move_frame, position
  const uint32_t ox = xpair(v.x), oz = xpair(v.z);
  RecQ q;
  if (L.k == 0) {
    // (bytes b0..b3 of P1's word, b4..b7 of P2's: guard0 guard1 move0 move1 | action0 action1 hitstun0 hitstun1)
    q.x = __builtin_amdgcn_perm(ox, v.x, 0x05010400u);
    q.y = __builtin_amdgcn_perm(ox, v.x, 0x07030602u);
    q.z = terminated;  // (truncated and the pad bytes: 0)
    q.w = v.y;
  } else {
    q.x = v.y;
    q.y = oz;
    q.z = v.z;
    q.w = (uint32_t)L.frame_count;
  }
  char* b = reinterpret_cast<char*>(rec) + 40u * r;
  *reinterpret_cast<RecQ*>(b + 16u * L.k) = q;
  if (L.k == 0) {
    const uint64_t rw = (uint64_t)__double_as_longlong(reward);
    *reinterpret_cast<uint2*>(b + 32u) = make_uint2((uint32_t)rw, (uint32_t)(rw >> 32));
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ uint32_t hash_action(uint64_t seed, uint64_t env, uint64_t t, uint32_t player) {
  return (uint32_t)(splitmix64(seed ^ (env * 0x9E3779B97F4A7C15ull) ^ ((t << 1) | player)) & 7u);
}

// ---------------------------------------------------------------------------
// one env-step: FootsiesEnv.step (FE:518-570) over the synced game's Fight tick
// (BC:201-220, 347-364) and, for a terminal arena, the auto-reset burst
// ---------------------------------------------------------------------------
// `next` is the next tick's action, loaded by the caller before this tick: it is made
// resident before this tick's first store.  Loads and stores share one in-order
// counter (vmcnt) on gfx9, so a wait for `next` placed after the stores (where the
// compiler would put it, at the loop latch) would also wait for every store of the
// tick to be acknowledged by memory (settle_w below).

// The fused loop's action rows, two ticks ahead, as loads the compiler does not track.  With the
// compiler's own load the row for tick t+1 had to be resident before tick t's stores, a wait that
// also drained tick t-1's stores (gfx9 counts loads and stores on one in-order vmcnt) and left one
// tick to cover the load.  Here the row for tick t+1 is issued at the top of tick t-1, and before
// tick t's stores the wave waits with vmcnt(11): at least 11 vector memory ops were issued after
// that load -- tick t-1's output stores (10 on every path of env_step: write_main's 7 plus reward,
// terminated, truncated) and tick t+2's load -- so the row is resident while those stores may
// still be in flight.  (Packed trajectories, PK: 2 stores per tick, so vmcnt(3).)  The loaded register is read by nothing but the wait statement, which copies
// the row out after the s_waitcnt; tools/check_async_loads.py checks on the assembly that no
// instruction touches a register between its load and its wait, and that on every path at least
// 11 vector memory instructions are issued between each row load and its wait
// (tests/test_async_loads.py).
__device__ __forceinline__ uint32_t row_load(const uint8_t* p) {
  uint32_t v;
  asm volatile("global_load_ubyte %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
template <int WAIT>
__device__ __forceinline__ void settle_w(uint32_t& next) {
  if constexpr (WAIT < 0) {
    asm volatile("" : "+v"(next));
  } else {
    // the in-flight register is read only by this statement, after the wait; the value the next
    // tick uses is a fresh register written here
    uint32_t ready;
    asm volatile("s_waitcnt vmcnt(%2)\n\tv_mov_b32 %0, %1" : "=v"(ready) : "v"(next), "n"(WAIT) : "memory");
    next = ready;
  }
}

// Time-sliced wave priority.  At C3's 65 536 arenas each SIMD holds two waves of the fused loop,
// one from block b and one from block b + 256 (256 CUs).  With equal priorities the sequencer
// favours the older wave, so it runs ~11 % ahead and finishes first, and the younger one runs its
// last ~10 % of ticks alone on the SIMD, where one wave cannot issue as fast as two
// (tools/timeline_probe.py: loop times 988 vs 1099 us of a 1000-tick launch, 17.9 vs 22.1 us of a
// 20-tick one).  Every tick each wave raises its priority in alternate 2^9 / 100 MHz = 5.1 us
// slices of the constant clock all CUs share, the two waves of a SIMD (wave slots of opposite
// parity) in opposite slices, so both progress at the same rate and finish together.
// (+4.8 % at 1000 ticks per launch, +3.4 % at 20; slices of 0.64 us: +0.4 %.)  With one wave per
// SIMD there is nothing to balance and the clock read only lengthens the lone wave's tick (-3.5 %
// at 32 768 arenas, profiles/r04d_ab32k.txt), so the launcher sets StepParams::prio only when the
// grid holds more waves than the device has SIMDs.
constexpr int kPrioSliceShift = 9;
__device__ __forceinline__ uint32_t prio_group() {
  return __builtin_amdgcn_s_getreg(4 /* HW_ID */ | (31 << 11)) & 1u;  // bit 0 of the wave slot
}
__device__ __forceinline__ void prio_slice(uint32_t grp) {
  const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime() ^ (grp << kPrioSliceShift);
  asm volatile("s_bitcmp1_b32 %0, %1\n\ts_cbranch_scc0 .Lprio_lo%=\n\ts_setprio 1\n\ts_branch .Lprio_end%=\n"
               ".Lprio_lo%=:\n\ts_setprio 0\n.Lprio_end%=:" :: "s"(now), "n"(kPrioSliceShift) : "scc");
}

// The burst leaves mostly constants in the lane (SetupBattleStart, STAND's ActionInfo).  Where
// the pending branch joins the tick, the compiler would materialize those constants in the join
// block under the full exec mask -- a dozen moves on every tick of every wave, pending or not.
// Made opaque here, they are produced inside the branch, in the registers the tick's own results
// occupy.
__device__ __forceinline__ void opaque_burst_results(Lane& L) {
  asm volatile("" : "+v"(L.f.x), "+v"(L.f.act), "+v"(L.f.frame), "+v"(L.f.vital), "+v"(L.f.guard), "+v"(L.f.hits),
               "+v"(L.f.buf), "+v"(L.f.rsv), "+v"(L.f.hold), "+v"(L.f.won), "+v"(L.f.hist));
  asm volatile("" : "+v"(L.ai), "+v"(L.cum), "+v"(L.pending), "+v"(L.has_term), "+v"(L.frame_count),
               "+v"(L.rec_count));
}

// Tick t + 1's request inputs, prepared at the end of tick t (the fused row loop at one wave per
// SIMD, StepParams::prefetch): UpdateInput (F:172-188) and IncrementActionFrame (F:140-166) of tick
// t + 1 depend only on its input -- resident once tick t has waited for the next row -- and on the
// fighter after tick t, so they run after tick t's stores, and the request-table entry and the
// continuing frame record are read then: the next tick's head starts with both resident instead of
// waiting for that dependent LDS round trip (a lone wave has no partner to issue in the wait).
// The C# order of tick t + 1 is unchanged: nothing between the end of tick t and UpdateInput of
// tick t + 1 (frameCount++, RecordInput) reads or writes what these phases touch.
struct Pre {
  InputEval e;
  uint32_t q;      // request-table entry (kTables.req_table[request_sel])
  int rec_cont;    // frame record if the action continues
  uint32_t keep;   // hasWon / an early return (request_sel's `keep`)
};
// The input a tick of this lane acts on, from its action row's byte (env_step's `in`, not stored)
template <int P2>
__device__ __forceinline__ uint32_t tick_input(const Lane& L, uint32_t a_own) {
  static_assert(P2 != kActors, "(the per-arena actors take env_step's own path)");
  if (L.k == 0 || P2 == FS_P2_EXTERNAL) return a_own;
  return P2 == FS_P2_BOT ? L.bin : 0u;
}
__device__ __forceinline__ void prepare_request(Lane& L, uint32_t in, Pre& pre) {
  pre.e = update_input(L.f, in, L.k ? kRelLut1 : kRelLut0);
  increment_action_frame(L.f, L.ai);
  pre.rec_cont = frame_record<false>(L.f);
  bool keep;
  const uint32_t sel = request_sel(L.f, pre.e, L.ai, keep);
  pre.keep = keep;
  pre.q = sT.req_table[sel];
}

template <int FM, int P2, int WAIT = -1, int TP = kTabLds, bool GEOM = false, bool PK = false, bool PF = false>
__device__ __forceinline__ void env_step(Lane& L, uint32_t a_own, const StepParams& p, uint32_t r, uint32_t& next,
                                         const Pre& pre = Pre{}, bool use_pre = false) {
  constexpr bool BOT = P2 == FS_P2_BOT;
  constexpr bool G = TP == kTabGlobal;  // the tables from global memory: a one-tick launch (k_step),
                                        // where no next tick reads L.ai
  const DevOutputs& o = p.out;
  const uint32_t k = L.k;
  const Actors ac{p.p1_bot != 0, p.p2_resets != 0, p.p2_noop != 0};
  if (L.pending) {  // FS_AUTORESET_NEXT_STEP: this step runs the reset burst only
    reset_burst<FM, P2, G>(L, true, ac);
    if constexpr (GEOM) {  // the round start's position (x, 0) and facing (F:123-124)
      L.f.y = 0.0f;
      L.f.flip = 0;
    }
    L.pending = false;
    L.has_term = false;
    L.cum = 0.0;
    L.ai = stand_info();  // the burst ends on STAND
    settle_w<WAIT>(next);
    if constexpr (PK) {
      write_packed(L, o.pk_lanes, r, k == 0 ? (uint32_t)L.frame_count : 0u);
      st_off(o.reward, 8 * r, 0.0);
    } else {
      write_main(L, o, r);
      st_off(o.reward, 8 * r, 0.0);  // per-arena outputs: both lanes store the same value (no divergent branch)
      st_off(o.terminated, r, (uint8_t)0);
      st_off(o.truncated, r, (uint8_t)0);
      if constexpr (G) {
        if (p.rec) write_record(L, p.rec, r, 0u, 0.0);
      }
    }
    opaque_burst_results(L);
    return;
  }
  // the actor inputs of this frame (TrainingManager.p1Input/p2Input, BC:383-447): a remote
  // actor's new action, or the input a bot computed after the last frame
  uint32_t in;
  if constexpr (P2 == kActors) {
    const bool mybot = k == 0 ? ac.p1_bot : L.p2bot;
    const bool idle = k == 1 && ac.p2_noop;
    L.act = (!mybot && !idle) ? a_own : L.act;
    in = mybot ? L.bin : (idle ? 0u : L.act);
  } else {
    if (k == 0 || P2 == FS_P2_EXTERNAL) L.act = a_own;
    in = (BOT && k == 1) ? L.bin : ((P2 == FS_P2_NOOP && k == 1) ? 0u : L.act);
  }
  const int guard_before = L.f.guard;  // guards of FE._current_state
  BotPre bpre;
  if constexpr (BOT) bpre = bot_prefetch<G>(L.bot, k);  // consumed by this tick's bot call, at its end
  L.frame_count++;
  if (L.rec_count < kMaxRecording) {  // RecordInput (BC:593-607)
    L.rec = in;
    L.rec_count++;
  }
  // the fighter's facing: the player's own, or flipped by a state load (general geometry)
  const uint32_t face = GEOM ? k ^ L.f.flip : k;
  InputEval e;
  int rec_cont;
  uint32_t rec_set;
  bool set;
  if (PF && use_pre) {  // prepared at the end of the previous tick (prepare_request; uniform per wave)
    e = pre.e;
    rec_cont = pre.rec_cont;
    set = apply_request(L.f, pre.q, pre.keep != 0, e, &rec_set);
  } else {
    e = update_input(L.f, in, face ? kRelLut1 : kRelLut0);
    const AInfo ai = L.ai;  // ActionInfo of f.act, re-read at the end of the previous tick
    increment_action_frame(L.f, ai);
    // the record if the action continues, read alongside the request entry; a
    // request that sets an action returns that action's frame-0 record
    rec_cont = frame_record<G>(L.f);
    set = update_action_request<G>(L.f, e, ai, &rec_set);
  }
  L.f.rec = set ? (int)rec_set : rec_cont;
  // One LDS round trip for everything the rest of the tick reads from the tables: my frame
  // record, the y half of the box-pair overlaps (records only, kTables.ybits) and the hit
  // resolution of the partner's record at its hit count (the record index and the hit count
  // cross the pair first).
  const RecGeo R = frame_rec<G>(face, (uint32_t)L.f.rec);
  const uint32_t o_rec = (uint32_t)xpair(L.f.rec);
  const uint32_t o_hits = (uint32_t)xpair(L.f.hits);
  static_assert(kNumFrameRecs <= 64, "ybits rows are 64 records wide");
  const uint32_t ym = tabs<G>().ybits[(o_rec << 6) | (uint32_t)L.f.rec];
  const U4 res = reinterpret_cast<const U4*>(tabs<G>().resolve)[__umul24(o_hits, (uint32_t)kNumFrameRecs) + o_rec];
  update_movement<FM>(L.f, R.push.z);
  update_boxes<FM>(L.f, R);
  RecY Y;
  if constexpr (GEOM) {
    Y = rec_y((uint32_t)L.f.rec);
    update_boxes_y<FM>(L.f, Y);
  }
  // the partner's hitbox half-widths (its own record's)
  const float o_hw0 = xpair(R.hit.z), o_hw1 = xpair(R.hit.w);
  push_character_vs_character<FM, GEOM>(L.f, k, GEOM ? Y.a.y : 0.0f);
  push_character_vs_background<FM, GEOM>(L.f);
  // consumed here, unconditionally, so the reads stay where they were issued (next to the
  // frame record) instead of being sunk into the collision's branch
  // (R.push too: a register of a load in flight that the allocator considers free is reused at
  // once, which forces a wait for the load)
  asm volatile("" ::"v"(R.push), "v"(R.hurt), "v"(o_hw0), "v"(o_hw1), "v"(res), "v"(ym));
  uint32_t ym_t = ym;
  if constexpr (GEOM) {  // the y half of BoxBase.Overlaps (F:17-25) from the boxes' y after the pushes
    const float o_hy0 = xpair(L.f.hy0), o_hy1 = xpair(L.f.hy1), o_hh0 = xpair(Y.b.w), o_hh1 = xpair(Y.c.y);
    const float hymax0 = fadd<FM>(o_hy0, o_hh0), hymax1 = fadd<FM>(o_hy1, o_hh1);  // partner's hitboxes
    const float uymax0 = fadd<FM>(L.f.uy0, Y.a.w), uymax1 = fadd<FM>(L.f.uy1, Y.b.y);  // my hurtboxes
    auto ov = [](float uy, float uymax, float hy, float hymax) { return (uint32_t)((uymax >= hy) & (uy <= hymax)); };
    ym_t = ov(L.f.uy0, uymax0, o_hy0, hymax0) | (ov(L.f.uy1, uymax1, o_hy0, hymax0) << 1) |
           (ov(L.f.uy0, uymax0, o_hy1, hymax1) << 2) | (ov(L.f.uy1, uymax1, o_hy1, hymax1) << 3);
  }
  hitbox_hurtbox_collision<FM>(L.f, k, R.hurt, o_hw0, o_hw1, res, ym_t);
  // the next tick's ActionInfo, issued now so its LDS latency hides behind the KO test, the
  // reward and the stores (only the same-step reset below changes the action again: to STAND)
  if constexpr (!G) L.ai = action_info<G>(L.f.act);
  // KO check (BC:212-213) and reward (FE:382-405), evaluated identically on both lanes: each
  // lane's flags (bit 0: vital 0, bit 1: guard dropped this tick; both fields are 0..3) cross
  // the pair once, then fl1 / fl2 are P1's / P2's
  const uint32_t my_fl = ((uint32_t)(L.f.vital - 1) >> 31) | (((uint32_t)(L.f.guard - guard_before) >> 31) << 1);
  const uint32_t o_fl = xpair(my_fl);
  const uint32_t any_fl = my_fl | o_fl;
  const bool over = (any_fl & 1u) != 0;
  double reward = 0.0;
  if (p.dense_reward) {
    // Only a guard drop or the round's end moves the f64 sums: on other ticks the reward is
    // 0.0 and `cum += 0.0` is exact (cum starts at +0.0 and a sum of nonzero terms is never -0.0).
    if (any_fl != 0) {
      const uint32_t fl1 = k == 0 ? my_fl : o_fl, fl2 = k == 0 ? o_fl : my_fl;
      if (fl1 & 2u) reward -= 0.3;
      if (fl2 & 2u) reward += 0.3;
      L.cum += reward;
      if (over) reward += (double)((fl2 & 1u) ? 1 : -1) - L.cum;
    }
  } else {
    const uint32_t fl2 = k == 0 ? o_fl : my_fl;
    reward = over ? ((fl2 & 1u) ? 1.0 : -1.0) : 0.0;
  }
  settle_w<WAIT>(next);
  if (over) {
    L.f.hist = 0;  // ChangeRoundState(KO): ClearInput (BC:296-299)
    L.f.hold = 0;
    if (p.autoreset_mode == FS_AUTORESET_SAME_STEP) {
      if constexpr (PK) write_packed(L, o.pk_final, r, k == 0 ? (uint32_t)L.frame_count : 0u);
      else write_final(L, o, r);
      reset_burst<FM, P2, G>(L, true, ac);
      if constexpr (GEOM) {
        L.f.y = 0.0f;
        L.f.flip = 0;
      }
      L.cum = 0.0;
      L.has_term = false;
      L.ai = stand_info();  // the burst ends on STAND
    } else {
      L.pending = true;
      L.has_term = true;
    }
  } else {
    if constexpr (BOT) {  // TrainingManager.Step -> RequestNextInput -> getNextAIInput
      const float x1 = xp1(L.f.x), x2 = xp2(L.f.x);
      const uint32_t p1_act = xp1((uint32_t)L.f.act);
      const uint32_t bi = bot_next_input<G>(L.bot, k, bot_distance<FM>(x1, x2), p1_act, bpre);
      L.bin = k == 1 ? bi : L.bin;
    } else if constexpr (P2 == kActors) {  // the same, for the per-arena actors
      const float x1 = xp1(L.f.x), x2 = xp2(L.f.x);
      const uint32_t p1_act = xp1((uint32_t)L.f.act), p2_act = xp2((uint32_t)L.f.act);
      actors_request<G>(L, ac, bot_distance<FM>(x1, x2), p1_act, p2_act);
    }
    L.has_term = false;
  }
  if constexpr (PK) {
    write_packed(L, o.pk_lanes, r, k == 0 ? (uint32_t)L.frame_count : (over ? 1u : 0u));
    st_off(o.reward, 8 * r, reward);  // identical on both lanes of the arena
  } else {
    write_main(L, o, r);
    st_off(o.reward, 8 * r, reward);  // identical on both lanes of the arena
    st_off(o.terminated, r, (uint8_t)(over ? 1 : 0));
    st_off(o.truncated, r, (uint8_t)0);
    if constexpr (G) {
      if (p.rec) write_record(L, p.rec, r, over ? 1u : 0u, reward);
    }
  }
  // all four words live until here (the tick reads three; see R.push above)
  if constexpr (!G) asm volatile("" ::"v"(L.ai));
}

// P1's observation features for the in-kernel actor (fs_policy.h), packed bf16x2:
// guard / 3 | move / 16 and move_frame / 55 | position / 4.6, the values write_obs stores
// (FE:339-358, 537-549) scaled by f32 reciprocals.
__device__ __forceinline__ void policy_features(const Lane& L, uint32_t& d0, uint32_t& d1) {
  int a = L.f.act;
  if (a == A_DEAD || a == A_WIN) a = A_STAND;
  const int mf = (a == A_STAND || a == A_FORWARD || a == A_BACKWARD) ? 0 : L.f.frame;
  d0 = pack_bf16x2((float)L.f.guard * (1.0f / 3.0f), (float)a * (1.0f / 16.0f));
  d1 = pack_bf16x2((float)mf * (1.0f / 55.0f), L.f.x * (1.0f / 4.6f));
}

// One fused launch over all arenas (k_step_n*, the rollout: state stays in registers between the
// p.n_steps ticks); the one-tick launch is step_one below.
// HASH draws the actions in-kernel from splitmix64 instead of reading action rows.
// POL samples P1's action every tick from the MLP actor (fs_policy.h); its MFMAs and lane
// exchanges need the whole wave, so lanes past the last arena stay in the loop (on a copy
// of arena 0 that they never store) unless their whole wave is idle.
template <int FM, int P2, bool FUSED, bool HASH, bool POL = false, bool GEOM = false, bool PK = false, bool PF = false>
__device__ __forceinline__ void step_body(const StepParams& p) {
  static_assert(!PK || (FUSED && !HASH && !POL), "packed trajectories: the fused row loop only");
  static_assert(!PF || (FUSED && !HASH && !POL && !GEOM && P2 != kActors), "request prefetch: the standard row loop");
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = l < 2 * p.n_envs;
  const int a = active ? l >> 1 : 0;
  const uint32_t k = l & 1;
  // This lane's action, software-pipelined one tick ahead: the load for tick t+1
  // is issued before tick t's output stores, so its wait does not drain them
  // (loads and stores retire in order on one vmcnt counter).
  const uint8_t* src = k == 0 ? p.p1 : p.p2;
  // which lanes read an action row: P1's unless the actor or a P1 bot plays it; P2's when the handle
  // has a remote P2 (kActors: per arena, so the row is read and ignored while the bot plays).  A
  // handle whose P2 is the bot or idle has no P2 rows at all (p.p2 is null).
  const bool p2_rows = P2 == FS_P2_EXTERNAL || (P2 == kActors && !p.p2_noop && !p.p2_resets);
  const bool reads = k == 0 ? (!POL && !(P2 == kActors && p.p1_bot)) : p2_rows;
  auto fetch = [&](int t) -> uint32_t {
    if (!reads) return 0u;
    if constexpr (HASH) {
      return hash_action(p.action_seed, p.arena_base + (uint64_t)a, p.t0 + (uint64_t)t, k);
    } else {
      return src[(uint32_t)t * (uint32_t)p.n_envs + (uint32_t)a];
    }
  };
  // the arena state and the first action are in flight while the block stages the tables
  Lane L;
  load_lane<P2>(L, p.st, a, k);
  if constexpr (GEOM) L.f.y = reinterpret_cast<const float*>(p.st.posy)[2 * a + (int)k];
  // the fused loop's rows: every lane loads (so the in-flight register is written by the load
  // alone); a lane without a row of its own reads P1's row 0, always valid in these launches,
  // and ignores it.  Rows 0 and 1 are both in flight while the block stages the tables.
  const int last = p.n_steps - 1;
  const uint8_t* own = reads ? src : p.p1;
  const uint32_t row_mul = reads ? (uint32_t)p.n_envs : 0u;
  auto issue = [&](int t) -> uint32_t { return row_load(own + (uint32_t)min(t, last) * row_mul + (uint32_t)a); };
  uint32_t next, row1 = 0;
  if constexpr (FUSED && !HASH && !POL) {
    next = issue(0);
    row1 = issue(1);
  } else {
    next = fetch(0);
  }
  if constexpr (POL) stage_policy(p.pol);
  if constexpr (FUSED) stage_tables<P2 == FS_P2_BOT || P2 == kActors>();
  if constexpr (POL) {
    if ((l & ~63) >= 2 * p.n_envs) return;  // the whole wave is past the last arena
  } else {
    if (!active) return;
  }
  L.ai = action_info<false>(L.f.act);
  if constexpr (POL) {
    const uint32_t row_step = (uint32_t)p.out_stride_steps * (uint32_t)p.n_envs;
    const uint32_t arena0 = (uint32_t)(l & ~63) >> 1;
    uint32_t d0, d1;
    policy_features(L, d0, d1);
    const PolicyWeights W = policy_weights();
    const uint32_t grp = prio_group();
    for (int t = 0; t < p.n_steps; t++) {
      const uint32_t act = next;
      next = fetch(min(t + 1, p.n_steps - 1));
      if (p.prio) prio_slice(grp);
      const PolicyOut po = policy_act(W, d0, d1, p.pol.seed, p.arena_base + arena0, p.t0 + (uint64_t)t);
      if (active) {
        const uint32_t row = (uint32_t)t * (uint32_t)p.n_envs + (uint32_t)a;
        if (k == 0) {
          if (p.pol.actions) p.pol.actions[row] = (uint8_t)po.action;
          if (p.pol.logp) p.pol.logp[row] = po.logp;
        }
        env_step<FM, P2, -1, kTabLds, GEOM>(L, k == 0 ? po.action : act & 7u, p, (uint32_t)t * row_step + (uint32_t)a,
                                            next);
      }
      policy_features(L, d0, d1);
    }
  } else if constexpr (FUSED) {
    const uint32_t row_step = (uint32_t)p.out_stride_steps * (uint32_t)p.n_envs;
    if constexpr (HASH) {
      const uint32_t grp = prio_group();
      for (int t = 0; t < p.n_steps; t++) {
        const uint32_t act = next;
        next = fetch(min(t + 1, p.n_steps - 1));
        if (p.prio) prio_slice(grp);
        env_step<FM, P2, -1, kTabLds, GEOM>(L, act & 7u, p, (uint32_t)t * row_step + (uint32_t)a, next);
      }
    } else {
      // Rows two ticks ahead, loaded and waited for as described at row_load, in two registers
      // that swap roles every tick (unrolled by two, so no register copy of a row in flight).
      // *_fl: a load in flight (read only by its wait), *_rd: the row once resident.  A load is
      // issued every tick (the last rows re-read the last one) so the wait counts hold, and the
      // last one in flight is waited for before the wave ends.  (Rows 0 and 1 were issued before
      // the table staging.)
      // (the wait count of settle_w: the vector memory ops every path issues between a row's load
      // and its wait -- one tick's output stores, 10 per-field or 2 packed, plus the next row load)
      constexpr int kRowWait = PK ? 3 : 11;
      uint32_t a_fl = next, b_fl = row1, a_rd, b_rd;
      asm volatile("s_waitcnt vmcnt(0)\n\tv_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=v"(a_rd), "=v"(b_rd)
                   : "v"(a_fl), "v"(b_fl) : "memory");
      const uint32_t grp = prio_group();
      // PF: each tick but the launch's first starts from the request prepared at the end of the
      // tick before it (prepare_request), from the row that tick made resident
      Pre pre{};
      bool have = false;
      int t = 0;
      for (; t < last; t += 2) {
        a_fl = issue(t + 2);
        if (p.prio) prio_slice(grp);
        env_step<FM, P2, kRowWait, kTabLds, GEOM, PK, PF>(L, reads ? a_rd & 7u : 0u, p,
                                                        (uint32_t)t * row_step + (uint32_t)a, b_fl, pre, have);
        b_rd = b_fl;
        if constexpr (PF) {
          prepare_request(L, tick_input<P2>(L, reads ? b_rd & 7u : 0u), pre);
          have = true;
        }
        b_fl = issue(t + 3);
        if (p.prio) prio_slice(grp);
        env_step<FM, P2, kRowWait, kTabLds, GEOM, PK, PF>(L, reads ? b_rd & 7u : 0u, p,
                                                        (uint32_t)(t + 1) * row_step + (uint32_t)a, a_fl, pre, PF);
        a_rd = a_fl;
        if constexpr (PF) {
          if (t + 2 <= last) prepare_request(L, tick_input<P2>(L, reads ? a_rd & 7u : 0u), pre);
        }
      }
      if (t == last) {  // an odd tick count: the last tick waits for a re-read of the last row
        a_fl = issue(t + 2);
        uint32_t b_last = b_fl;  // (b_fl itself stays the in-flight value for the final wait)
        env_step<FM, P2, kRowWait, kTabLds, GEOM, PK, PF>(L, reads ? a_rd & 7u : 0u, p,
                                                        (uint32_t)t * row_step + (uint32_t)a, b_last, pre, have);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::"v"(a_fl), "v"(b_fl) : "memory");  // no load outlives the wave
    }
  }
  if (active) {
    store_lane<P2>(L, p.st, a);
    if constexpr (GEOM) reinterpret_cast<float*>(p.st.posy)[2 * a + (int)k] = L.f.y;
  }
}

// The one-tick launch (fs_step, fs_step_masked: the VectorEnv.step path).  Nothing is amortized
// over ticks here, so the kernel is one dependent chain of memory round trips, and its prologue
// is arranged to keep that chain short:
// * every kernel argument the prologue needs is brought into SGPRs at once (one scalar-memory
//   round trip; the compiler otherwise issued the state pointers' loads in two batches and the
//   mask pointer's after the first vector loads had been waited for), and the block size is the
//   launch constant kBlock rather than the dispatch packet's;
// * the action row of the lane's player is selected between two SGPR pointers in registers (a
//   per-lane `k ? p2 : p1` on the argument struct was compiled into a vector load of the pointer
//   from the kernel-argument segment, waited for together with the state loads, before the
//   action byte could be loaded), so the action byte, the mask byte and the arena state are in
//   flight together;
// * the tick's first table lookup, the ActionInfo of each fighter's action, comes from a copy of
//   the 17-entry ActionInfo table that the wave's lanes 0-16 load alongside the state (lane j
//   entry j) and a ds_bpermute by action index: an LDS-crossbar exchange instead of a dependent
//   global-memory round trip after the state arrives.  Every lane is still active at that point
//   (the exchange reads other lanes' registers), and lanes past the last arena leave after it.
__device__ uint8_t kOneByte = 1;  // (global memory, so the select below stays a global load)
template <int FM, int P2>
__device__ __forceinline__ void step_one(const StepParams& p) {
  const uint8_t* q1 = p.p1;
  const uint8_t* q2 = p.p2;
  const uint8_t* qm = p.active;
  const int n_envs = p.n_envs, inl_n = p.inl_n;
  // (inputs only: the pointers keep their global-memory provenance; and the two row pointers each
  // have a use of their own here, so `k ? q2 : q1` stays a register select)
  const int geom = p.geom;
  asm volatile("" ::"s"(p.st.pos), "s"(p.st.hist), "s"(p.st.fpk), "s"(p.st.aw), "s"(p.st.cum), "s"(q1), "s"(q2),
               "s"(qm), "s"(n_envs), "s"(inl_n), "s"(geom));
  const int l = blockIdx.x * kBlock + threadIdx.x;
  const bool active = l < 2 * n_envs;
  const int a = active ? l >> 1 : 0;
  const uint32_t k = l & 1;
  // the two ActionInfo words the tick reads (frame count / loop start, cancel window), lane j of
  // the wave holding action j's
  const uint32_t lane = threadIdx.x & 63u;
  const uint2 tab = reinterpret_cast<const uint2*>(kTables.action)[2u * min(lane, (uint32_t)kNumActions - 1u)];
  Lane L;
  load_lane<P2>(L, p.st, a, k);
  // this lane's input: host inputs in the kernel arguments (a few arenas), else its player's row
  // (P1's unless a P1 bot plays; P2's when the handle has a remote P2)
  const bool p2_rows = P2 == FS_P2_EXTERNAL || (P2 == kActors && !p.p2_noop && !p.p2_resets);
  const bool reads = k == 0 ? !(P2 == kActors && p.p1_bot) : p2_rows;
  const uint8_t* q = k == 0 ? q1 : q2;
  uint32_t in = 0;
  if (inl_n) in = (p.inl[k][(uint32_t)a >> 2] >> (8u * ((uint32_t)a & 3u))) & 0xffu;
  else if (reads) in = q[a];
  // fs_step_masked's byte, or a constant 1 (a load either way: no branch ahead of the state's use)
  const uint32_t on = *(qm ? qm + a : &kOneByte);
  // ActionInfo of the fighter's action, from lane L.f.act of this wave (all lanes active here)
  const int src = L.f.act << 2;
  L.ai.x = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)tab.x);
  L.ai.y = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)tab.y);
  L.ai.z = L.ai.w = 0u;  // (the cancel mask and padding: not read by the tick)
  if (!active || !on) return;
  uint32_t none = 0;
  if (geom) {  // (general geometry: position.y, read after the branch; off the common path)
    float* py = reinterpret_cast<float*>(p.st.posy) + 2 * a + (int)k;
    L.f.y = *py;
    env_step<FM, P2, -1, kTabGlobal, true>(L, in & 7u, p, (uint32_t)a, none);
    store_lane<P2>(L, p.st, a);
    *py = L.f.y;
  } else {
    env_step<FM, P2, -1, kTabGlobal>(L, in & 7u, p, (uint32_t)a, none);
    store_lane<P2>(L, p.st, a);
  }
}

template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step(StepParams p) {
  step_one<FM, P2>(p);
}

// Each fused kernel holds the standard tick and the general-geometry one (StepParams::geom,
// uniform over the launch) as two loops: the standard loop carries none of the y state.
template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n(StepParams p) {
  if (p.geom) step_body<FM, P2, true, false, false, true>(p);
  else step_body<FM, P2, true, false>(p);
}

// fs_step_n_packed: the row loop of k_step_n storing packed trajectory records
template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n_packed(StepParams p) {
  if (p.geom) step_body<FM, P2, true, false, false, true, true>(p);
  else step_body<FM, P2, true, false, false, false, true>(p);
}

// The same row loops with each tick's request prepared at the end of the tick before
// (StepParams::prefetch; one wave per SIMD).  Kernels of their own: the prepared request stays live
// across the loop's back edge, and in a shared kernel its registers would lower the standard loop's
// occupancy too (132 VGPRs instead of 122: three waves per SIMD instead of four).
template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n_pf(StepParams p) {
  step_body<FM, P2, true, false, false, false, false, true>(p);
}
template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n_packed_pf(StepParams p) {
  step_body<FM, P2, true, false, false, false, true, true>(p);
}

template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n_hashed(StepParams p) {
  if (p.geom) step_body<FM, P2, true, true, false, true>(p);
  else step_body<FM, P2, true, true>(p);
}

template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n_policy(StepParams p) {
  if (p.geom) step_body<FM, P2, true, false, true, true>(p);
  else step_body<FM, P2, true, false, true>(p);
}

// FootsiesEnv.reset (FE:482-515) / RESET (BC:143-146) / game start (BC:105-128), every handle
// kind through the per-arena actor logic (off the throughput path).
template <int FM>
__global__ __launch_bounds__(256) void k_reset(ResetParams p) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  stage_tables();
  if (l >= 2 * p.n_envs) return;
  const int a = l >> 1;
  const uint32_t k = l & 1;
  if (!p.init && p.mask && !p.mask[a]) return;
  const Actors ac{p.p1_bot != 0, p.p2_mode == FS_P2_BOT, p.p2_mode == FS_P2_NOOP};
  Lane L;
  if (p.init) {  // `new Fighter()` defaults (F:73-112), `new BattleAI()`, round state Stop
    L.k = k;
    L.f.x = 0.0f;
    L.f.hist = 0;
    L.f.act = A_STAND;
    L.f.frame = L.f.stun = L.f.vital = L.f.guard = L.f.hits = L.f.hold = 0;
    L.f.buf = L.f.rsv = NONE;
    L.f.in_back = L.f.prox = L.f.won = false;
    L.f.flip = 0;
    L.f.y = 0.0f;
    L.frame_count = 0;
    L.rec_count = L.rec = L.act = L.bin = 0;
    L.pending = false;
    L.has_term = true;
    L.cum = 0.0;
    L.p2bot = p.p2_mode == FS_P2_BOT;
    L.rng = rng_init((int32_t)(uint32_t)(p.base_seed + p.arena_base + (uint64_t)a));
    L.fb.mplan = L.fb.midx = L.fb.aplan = L.fb.aidx = L.fb.prev_opp = 0;
    L.fb.prev_dist = 0.0f;
    L.fb.ready = false;
  } else {
    load_lane<kActors>(L, p.st, a, k);
    L.f.y = reinterpret_cast<const float*>(p.st.posy)[l];
  }
  if (p.seeds) L.rng = rng_init((int32_t)(uint32_t)p.seeds[a]);  // SEED (BC:170-173)
  if (p.flags == FS_RESET_SEED_ONLY) {
    store_lane<kActors>(L, p.st, a);
    reinterpret_cast<float*>(p.st.posy)[l] = L.f.y;
    return;
  }
  const bool hard = p.init || p.flags == FS_RESET_HARD || !L.has_term;
  if (L.pending) {  // finish the burst Unity ran after the terminal frame
    reset_burst<FM, kActors>(L, true, ac);
    L.pending = false;
    L.f.y = 0.0f;  // the round start's position (x, 0) and facing (F:123-124)
    L.f.flip = 0;
  }
  if (hard) {
    reset_burst<FM, kActors>(L, false, ac);
    L.f.y = 0.0f;
    L.f.flip = 0;
  }
  L.cum = 0.0;
  L.has_term = p.init ? true : false;
  write_main(L, p.out, a);
  if (k == 0) {
    p.out.reward[a] = 0.0;
    p.out.terminated[a] = 0;
    p.out.truncated[a] = 0;
  }
  store_lane<kActors>(L, p.st, a);
  reinterpret_cast<float*>(p.st.posy)[l] = L.f.y;
}

// P2_BOT (BC:158-167): P2's actor of the masked arenas becomes the bot (bot = 1) or the remote actor
__global__ __launch_bounds__(256) void k_set_p2(DevState st, int bot, const uint8_t* mask, int n) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n || (mask && !mask[a])) return;
  const uint32_t h = (uint32_t)st.aw[a].y;
  st.aw[a].y = (int)((h & ~(1u << 29)) | ((uint32_t)(bot != 0) << 29));
}

// synthetic action stream (fs_hash_actions), one thread per (step, arena)
__global__ __launch_bounds__(256) void k_hash_actions(int n_envs, int n_steps, uint64_t seed, uint64_t t0,
                                                       uint64_t arena_base, uint8_t* p1, uint8_t* p2) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)n_envs * n_steps) return;
  const uint64_t env = arena_base + idx % (size_t)n_envs, k = idx / (size_t)n_envs;
  p1[idx] = (uint8_t)hash_action(seed, env, t0 + k, 0);
  if (p2) p2[idx] = (uint8_t)hash_action(seed, env, t0 + k, 1);
}

// a bot word <-> its canonical fields (fs_arena_state): queues as (plan id, dequeued count),
// plan -1 = empty; the FightState as (distance, raw opponent actionID)
struct BotFields {
  int32_t move_plan, move_index, attack_plan, attack_index;
  float prev_distance;
  int32_t prev_opponent_action;
  uint8_t ready, input;
};
__device__ __forceinline__ BotFields bot_export(uint2 w) {
  uint32_t input;
  const FullBot b = unpack_bot(w, input);
  BotFields f;
  f.move_plan = b.mplan ? (int32_t)b.mplan - 1 : -1;
  f.move_index = b.mplan ? (int32_t)b.midx : 0;
  f.attack_plan = b.aplan ? (int32_t)b.aplan - 1 : -1;
  f.attack_index = b.aplan ? (int32_t)b.aidx : 0;
  f.prev_distance = b.ready ? b.prev_dist : 0.0f;  // no FightState yet: canonical zeros
  f.prev_opponent_action = b.ready ? kActionId[b.prev_opp] : 0;
  f.ready = b.ready;
  f.input = (uint8_t)input;
  return f;
}

// canonical export (fs_get_state / fs_get_env_state)
__global__ __launch_bounds__(256) void k_get_state(DevState st, fs_arena_state* dst, fs_env_state* env, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Arena A;
  load_arena(A, st, i);
  if (dst) {
    fs_arena_state s;
    for (int k = 0; k < 2; k++) {
      const Fighter& f = k == 0 ? A.f0 : A.f1;
      fs_fighter_state& g = s.f[k];
      g.position_x = f.x;
      g.action_id = kActionId[f.act];
      g.action_frame = f.frame;
      g.hit_count = f.hits;
      g.hitstun = f.stun;
      g.vital = f.vital;
      g.guard = f.guard;
      g.buffer_action_id = f.buf == NONE ? -1 : kActionId[f.buf];
      g.reserve_action_id = f.rsv == NONE ? -1 : kActionId[f.rsv];
      g.input_dir_history = raw_hist(f.hist, k ^ (int)f.flip);  // (the history is kept facing-relative)
      g.attack_hold = f.hold;
      g.is_input_backward = f.in_back;
      g.is_reserve_proximity_guard = f.prox;
      g.has_won = f.won;
      g.facing_flipped = (uint8_t)f.flip;
      g.position_y = f.y;
    }
    s.frame_count = A.frame_count;
    s.recording_count = (int32_t)A.rec_count;
    s.recording_last[0] = (uint8_t)A.rec1;
    s.recording_last[1] = (uint8_t)A.rec2;
    s.actor_input[0] = (uint8_t)A.act1;
    s.actor_input[1] = (uint8_t)A.act2;
    s.reset_pending = A.pending;
    s.has_terminated = A.has_term;
    s.pad0[0] = s.pad0[1] = 0;
    s.cumulative_reward = A.cum;
    s.rng[0] = A.rng.x;
    s.rng[1] = A.rng.y;
    s.rng[2] = A.rng.z;
    s.rng[3] = A.rng.w;
    const BotFields b2 = bot_export(A.bw[1]), b1 = bot_export(A.bw[0]);
    s.move_plan = b2.move_plan;
    s.move_index = b2.move_index;
    s.attack_plan = b2.attack_plan;
    s.attack_index = b2.attack_index;
    s.prev_distance = b2.prev_distance;
    s.prev_opponent_action = b2.prev_opponent_action;
    s.p2_bot = A.p2bot;
    s.bot_ready[0] = b1.ready;
    s.bot_ready[1] = b2.ready;
    s.bot_input[0] = b1.input;
    s.bot_input[1] = b2.input;
    s.pad1[0] = s.pad1[1] = s.pad1[2] = 0;
    s.p1_move_plan = b1.move_plan;
    s.p1_move_index = b1.move_index;
    s.p1_attack_plan = b1.attack_plan;
    s.p1_attack_index = b1.attack_index;
    s.p1_prev_distance = b1.prev_distance;
    s.p1_prev_opponent_action = b1.prev_opponent_action;
    dst[i] = s;
  }
  if (env) {
    fs_env_state e;
    e.p1Vital = A.f0.vital;
    e.p2Vital = A.f1.vital;
    e.p1Guard = A.f0.guard;
    e.p2Guard = A.f1.guard;
    e.p1Move = kActionId[A.f0.act];
    e.p1MoveFrame = A.f0.frame;
    e.p2Move = kActionId[A.f1.act];
    e.p2MoveFrame = A.f1.frame;
    e.p1Position = A.f0.x;
    e.p2Position = A.f1.x;
    e.globalFrame = A.frame_count;
    e.p1MostRecentAction = A.rec_count > 0 ? (int32_t)A.rec1 : 0;
    e.p2MostRecentAction = A.rec_count > 0 ? (int32_t)A.rec2 : 0;
    e.p1Hitstun = A.f0.stun;
    e.p2Hitstun = A.f1.stun;
    env[i] = e;
  }
}

__device__ __forceinline__ int action_index_of(int32_t id) {
  for (int a = 0; a < kNumActions; a++)
    if (kActionId[a] == id) return a;
  return -1;
}

__device__ __forceinline__ uint2 bot_import(int32_t mp, int32_t mi, int32_t ap, int32_t ai, float pd, int32_t po,
                                           uint8_t ready, uint8_t input) {
  FullBot b;
  b.mplan = mp < 0 ? 0u : (uint32_t)mp + 1;
  b.midx = mp < 0 ? 0u : (uint32_t)mi;
  b.aplan = ap < 0 ? 0u : (uint32_t)ap + 1;
  b.aidx = ap < 0 ? 0u : (uint32_t)ai;
  b.prev_dist = pd;
  b.prev_opp = (uint32_t)action_index_of(po);
  b.ready = ready != 0;
  return pack_bot(b, input & 7u);
}

__global__ __launch_bounds__(256) void k_set_state(DevState st, const fs_arena_state* src, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fs_arena_state s = src[i];
  Arena A;
  for (int k = 0; k < 2; k++) {
    const fs_fighter_state& g = s.f[k];
    Fighter& f = k == 0 ? A.f0 : A.f1;
    f.x = g.position_x;
    f.y = g.position_y;
    f.flip = g.facing_flipped & 1u;
    f.act = action_index_of(g.action_id);
    f.frame = g.action_frame;
    f.hits = g.hit_count;
    f.stun = g.hitstun;
    f.vital = g.vital;
    f.guard = g.guard;
    f.buf = g.buffer_action_id < 0 ? NONE : action_index_of(g.buffer_action_id);
    f.rsv = g.reserve_action_id < 0 ? NONE : action_index_of(g.reserve_action_id);
    f.hist = split_hist(g.input_dir_history, k ^ (int)f.flip);
    f.hold = g.attack_hold;
    f.in_back = g.is_input_backward;
    f.prox = g.is_reserve_proximity_guard;
    f.won = g.has_won;
  }
  A.frame_count = s.frame_count;
  A.rec_count = (uint32_t)s.recording_count;
  A.rec1 = s.recording_last[0] & 7;
  A.rec2 = s.recording_last[1] & 7;
  A.act1 = s.actor_input[0] & 7;
  A.act2 = s.actor_input[1] & 7;
  A.pending = s.reset_pending;
  A.has_term = s.has_terminated;
  A.cum = s.cumulative_reward;
  A.rng = make_uint4(s.rng[0], s.rng[1], s.rng[2], s.rng[3]);
  A.p2bot = s.p2_bot != 0;
  A.bw[1] = bot_import(s.move_plan, s.move_index, s.attack_plan, s.attack_index, s.prev_distance,
                       s.prev_opponent_action, s.bot_ready[1], s.bot_input[1]);
  A.bw[0] = bot_import(s.p1_move_plan, s.p1_move_index, s.p1_attack_plan, s.p1_attack_index, s.p1_prev_distance,
                       s.p1_prev_opponent_action, s.bot_ready[0], s.bot_input[0]);
  store_arena(A, st, i);
}

#include "fs_arena1.h"

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline dim3 grid_for(int n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

// Which kernel runs a fused launch with action rows.  The two-lane kernel needs two waves per SIMD
// to hide its LDS round trips, and has them from 32 768 arenas on; the one-lane kernel issues ~18 %
// fewer instructions per arena-tick but needs twice the arenas for the same waves: with one wave
// per SIMD (65 536 arenas, C3) it exposes the tick's dependent LDS reads and runs 16-18 % slower;
// from two waves per SIMD (131 072 arenas) on it matches the two-lane kernel with a remote P2 and
// beats it by 12-25 % with the scripted bot.  So the one-lane kernel takes the
// launches with at least two of its waves per SIMD -- except packed launches with a remote P2 from
// four of them on (262 144 arenas), where the two-lane packed kernel at 4 resident waves per SIMD is
// ahead (+4.3 % at 262 144, +1.4 % at 524 288; 131 072: one lane +2.1 %; profiles/r05l_ab_lanes_*.txt,
// r05m_ab_lanes_524288.txt); the per-field two-lane kernel, with its eight stores per tick, is not
// (7.2e10 vs 7.8-7.9e10 at 262 144).
// FOOTSIES_FUSED_LANES=1 / 2 forces one kernel (A/B timing, and the parity suite runs both).
static int simd_count() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;  // MI355X
  return 4 * cus;
}
static bool fused_one_lane(int n_envs, int variant, bool packed) {
  static const int forced = [] {
    const char* e = getenv("FOOTSIES_FUSED_LANES");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  if (forced) return forced == 1;
  static const int64_t threshold = 2 * 64 * (int64_t)simd_count();
  if (packed && variant == FS_P2_EXTERNAL) return n_envs >= threshold && n_envs < 2 * threshold;
  return n_envs >= threshold;
}

// Whether a fused launch with `lanes` lanes (two per arena, or one for the one-lane kernel) holds
// more than one wave per SIMD, the case prio_slice is for.  FOOTSIES_PRIO=0 / 1 forces it off / on
// (A/B timing).
static int prio_forced() {  // 0: not forced, 1: off, 2: on
  static const int forced = [] {
    const char* e = getenv("FOOTSIES_PRIO");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' + 1 : 0;
  }();
  return forced;
}
static bool waves_above_simds(int64_t lanes) {
  if (prio_forced()) return prio_forced() == 2;
  static const int simds = simd_count();
  return (lanes + 63) / 64 > simds;
}
static bool two_waves_per_simd(int n_envs) { return waves_above_simds(2 * (int64_t)n_envs); }
// The one-lane kernels: the slicing pays at two waves per SIMD (131 072 arenas: +4.4 % / +4.9 % remote
// P2, +4.1 % / +7.1 % bot, per-field / packed) and costs the remote-P2 case at four (262 144: -2.3 %,
// bot +3.3 %; profiles/r05g_ab_onelane_prio_131k.txt, r05h_ab_onelane_prio_*.txt), so only there.
static bool one_lane_prio(int n_envs) {
  if (prio_forced()) return prio_forced() == 2;
  static const int simds = simd_count();
  const int64_t waves = ((int64_t)n_envs + 63) / 64;
  return waves > simds && waves <= 2 * (int64_t)simds;
}

// Whether a two-lane fused row launch prepares each tick's request at the end of the tick before
// (Pre / prepare_request): at one wave per SIMD, where no partner wave issues in that LDS wait
// (DESIGN.md section 5); same-step auto-reset only (no tick is a next-step reset burst).
// FOOTSIES_PREFETCH=0 / 1 forces it off / on (A/B timing, and the parity suite runs both).
// (row_launch: a fused launch over action rows -- not the in-kernel actor's, not hashed actions)
static bool request_prefetch(bool row_launch, int autoreset_mode, bool geom, int n_steps, int n_envs) {
  static const int forced = [] {
    const char* e = getenv("FOOTSIES_PREFETCH");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' + 1 : 0;
  }();
  if (!row_launch || autoreset_mode != FS_AUTORESET_SAME_STEP || geom || n_steps < 2) return false;
  if (forced) return forced == 2;
  return !two_waves_per_simd(n_envs);
}

template <int FM, int P2>
static void launch_step_p2(const StepParams& p_in, hipStream_t s) {
  const dim3 grid = grid_for(2 * p_in.n_envs), block(kBlock);
  StepParams p = p_in;
  p.prio = two_waves_per_simd(p.n_envs);
  p.prefetch = P2 != kActors && request_prefetch(!p.pol.w1 && p.p1, p.autoreset_mode, p.geom, p.n_steps, p.n_envs);
  if (p.pol.w1) hipLaunchKernelGGL((k_step_n_policy<FM, P2>), grid, block, 0, s, p);
  else if (p.out.pk_lanes) {  // (rows: fs_api checks)
    if constexpr (P2 != kActors) {
      if (!p.geom && fused_one_lane(p.n_envs, P2, true)) {
        p.prio = one_lane_prio(p.n_envs);
        hipLaunchKernelGGL((k_step_n1_packed<FM, P2>), grid_for(p.n_envs), block, 0, s, p);
        return;
      }
    }
    if constexpr (P2 != kActors) {
      if (p.prefetch) {
        hipLaunchKernelGGL((k_step_n_packed_pf<FM, P2>), grid, block, 0, s, p);
        return;
      }
    }
    hipLaunchKernelGGL((k_step_n_packed<FM, P2>), grid, block, 0, s, p);
  }
  else if (!p.p1) hipLaunchKernelGGL((k_step_n_hashed<FM, P2>), grid, block, 0, s, p);
  else if (p.n_steps == 1) hipLaunchKernelGGL((k_step<FM, P2>), grid, block, 0, s, p);
  else if constexpr (P2 != kActors) {
    // (the one-lane kernel has no general-geometry tick: a geom launch takes the two-lane one)
    if (!p.geom && fused_one_lane(p.n_envs, P2, false)) {
      p.prio = one_lane_prio(p.n_envs);
      hipLaunchKernelGGL((k_step_n1<FM, P2>), grid_for(p.n_envs), block, 0, s, p);
    } else if (p.prefetch) {
      hipLaunchKernelGGL((k_step_n_pf<FM, P2>), grid, block, 0, s, p);
    } else {
      hipLaunchKernelGGL((k_step_n<FM, P2>), grid, block, 0, s, p);
    }
  } else {
    hipLaunchKernelGGL((k_step_n<FM, P2>), grid, block, 0, s, p);
  }
}

template <int FM>
static hipError_t launch_step_fm(const StepParams& p, int variant, hipStream_t s) {
  switch (variant) {
    case FS_P2_EXTERNAL: launch_step_p2<FM, FS_P2_EXTERNAL>(p, s); break;
    case FS_P2_BOT: launch_step_p2<FM, FS_P2_BOT>(p, s); break;
    case kActors: launch_step_p2<FM, kActors>(p, s); break;
    default: launch_step_p2<FM, FS_P2_NOOP>(p, s); break;
  }
  return hipGetLastError();
}

hipError_t launch_step(const StepParams& p, int float_mode, int variant, hipStream_t s) {
  return float_mode == FS_FLOAT_DOUBLE ? launch_step_fm<FS_FLOAT_DOUBLE>(p, variant, s)
                                       : launch_step_fm<FS_FLOAT_STRICT32>(p, variant, s);
}

// The kernel launch_step_p2 runs for a launch of this shape, as rocprofv3 names it (fs_step_kernel).
const char* step_kernel_name(bool policy, bool hashed, int n_steps, int n_envs, int float_mode, int variant, bool geom,
                             bool packed, int autoreset_mode) {
  static thread_local char buf[64];
  const bool one = !policy && !hashed && variant != kActors && !geom && fused_one_lane(n_envs, variant, packed);
  const bool pf = !one && variant != kActors && request_prefetch(!policy && !hashed, autoreset_mode, geom, n_steps, n_envs);
  const char* k = policy ? "k_step_n_policy" : packed ? (one ? "k_step_n1_packed" : pf ? "k_step_n_packed_pf" : "k_step_n_packed")
                : hashed ? "k_step_n_hashed" : n_steps == 1 ? "k_step" : one ? "k_step_n1" : pf ? "k_step_n_pf" : "k_step_n";
  snprintf(buf, sizeof buf, "fsk::%s<%d, %d>", k, float_mode == FS_FLOAT_DOUBLE ? 1 : 0, variant);
  return buf;
}

hipError_t launch_reset(const ResetParams& p, int float_mode, hipStream_t s) {
  if (float_mode == FS_FLOAT_DOUBLE)
    hipLaunchKernelGGL(k_reset<FS_FLOAT_DOUBLE>, grid_for(2 * p.n_envs), dim3(kBlock), 0, s, p);
  else
    hipLaunchKernelGGL(k_reset<FS_FLOAT_STRICT32>, grid_for(2 * p.n_envs), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_set_p2(const DevState& st, int bot, const uint8_t* mask, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_set_p2, grid_for(n), dim3(kBlock), 0, s, st, bot, mask, n);
  return hipGetLastError();
}

hipError_t launch_hash_actions(int n_envs, int n_steps, uint64_t seed, uint64_t t0, uint64_t arena_base, uint8_t* p1,
                               uint8_t* p2, hipStream_t s) {
  const size_t total = (size_t)n_envs * n_steps;
  hipLaunchKernelGGL(k_hash_actions, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n_envs,
                     n_steps, seed, t0, arena_base, p1, p2);
  return hipGetLastError();
}

hipError_t launch_get_state(const DevState& st, fs_arena_state* dst, fs_env_state* env, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_get_state, grid_for(n), dim3(kBlock), 0, s, st, dst, env, n);
  return hipGetLastError();
}

hipError_t launch_set_state(const DevState& st, const fs_arena_state* src, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_set_state, grid_for(n), dim3(kBlock), 0, s, st, src, n);
  return hipGetLastError();
}

}  // namespace fsk
