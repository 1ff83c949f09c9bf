// fs_kernels.hip -- HIP kernels for gfx950 (MI355X): one lane = one FOOTSIES arena.
//
// A Fight tick of the reference (BattleCore.FixedUpdate Fight branch ->
// UpdateFightState, Assets/Script/BattleCore.cs:201-220, 347-364) is restated
// over a bit-packed, struct-of-arrays arena state that lives in HBM:
//
//   load (5 coalesced 8/16-B vectors per lane) -> tick in registers -> store
//
// Frame data is the dense per-(action, frame) form generated into fs_tables.h
// (window scans of ActionData.cs:87-168 resolved offline).  The 180-deep input
// histories (Fighter.cs:98-101) are replaced by a 16-frame Left/Right shift
// register plus a saturating attack-hold counter: the reference only ever
// reads input[0..16] for dashes (Fighter.cs:585-635, dashAllowFrame 9) and
// "attack held on input[1..59]" for the charge special (Fighter.cs:569-583).
//
// Float arithmetic follows the C# expression order with every binary32
// operation rounded (__fadd_rn/__fmul_rn; the file is also built with
// -ffp-contract=off) or, in FS_FLOAT_DOUBLE mode, with binary64 temporaries.
//
// Paths: BC = Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs,
// AI = Assets/Script/BattleAI.cs, FE = footsies-gym/footsies_gym/envs/footsies.py.
#include <hip/hip_runtime.h>

#include "fs_internal.h"
#include "fs_tables.h"

#pragma clang fp contract(off)

namespace fsk {

constexpr int NONE = 31;  // empty buffer / reserve slot
constexpr uint32_t IN_LEFT = 1, IN_RIGHT = 2, IN_ATTACK = 4;

// ---------------------------------------------------------------------------
// frame data staged in LDS.  Every lookup of the tick (action info -> row ->
// box / velocity / cancel records) is a dependent, lane-divergent load; from
// LDS it costs ~tens of cycles instead of an L1/L2 round trip.  ~4.3 KB per
// block, copied once per launch by all threads of the block.
// ---------------------------------------------------------------------------
struct Tables {
  ActionInfo action[kNumActions];
  uint32_t rows[kNumRows];
  float4 rects[kNumRects];
  float vels[kNumVels];
  uint32_t hitsets[kNumHitSets];
  uint32_t hurtsets[kNumHurtSets];
  uint32_t cancel[kNumCancelMasks];
  AttackInfo attacks[4];
};
__shared__ Tables sT;

// all threads of the block must call this before any early return
__device__ __forceinline__ void stage_tables() {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int i = t; i < kNumRows; i += nt) sT.rows[i] = kRows[i];
  for (int i = t; i < kNumActions; i += nt) sT.action[i] = kActionInfo[i];
  for (int i = t; i < kNumRects; i += nt) sT.rects[i] = kRects[i];
  for (int i = t; i < kNumVels; i += nt) sT.vels[i] = kVels[i];
  for (int i = t; i < kNumHitSets; i += nt) sT.hitsets[i] = kHitSets[i];
  for (int i = t; i < kNumHurtSets; i += nt) sT.hurtsets[i] = kHurtSets[i];
  for (int i = t; i < kNumCancelMasks; i += nt) sT.cancel[i] = kCancelMasks[i];
  for (int i = t; i < 4; i += nt) sT.attacks[i] = kAttacks[i];
  __syncthreads();
}

// ---------------------------------------------------------------------------
// packed fighter word (u64), one per fighter in DevState::fpk
//   [0,5) action idx | [5,14) action frame | [14,19) hitstun | [19,21) vital |
//   [21,23) guard | [23,25) hit count | [25,30) buffer idx | [30,35) reserve idx |
//   35 isInputBackward | 36 isReserveProximityGuard | 37 hasWon | [38,44) attack hold
// arena header word (DevState::aw.y)
//   [0,15) recording count | [15,18) rec P1 | [18,21) rec P2 | [21,24) actor P1 |
//   [24,27) actor P2 | 27 reset pending | 28 has_terminated
// bot word (DevState::bot.x)
//   [0,3) move plan+1 (0 = empty) | [3,10) move index | [10,13) attack plan+1 |
//   [13,20) attack index | [20,25) previous FightState opponent action idx
// ---------------------------------------------------------------------------

struct Fighter {
  float x;
  uint32_t hist;  // raw Left/Right bits of input[0..15]
  int act, frame, stun, vital, guard, hits, buf, rsv, hold;
  bool in_back, prox, won;
  // boxes of this tick (UpdateBoxes, F:671-697), x only: y == rect.y since position.y == 0
  uint32_t hitset, hurtset;
  int push_rect;
  float hx0, hx1, ux0, ux1, px;
};

struct Arena {
  Fighter f0, f1;
  int frame_count;
  uint32_t rec_count, rec1, rec2, act1, act2;
  bool pending, has_term;
  double cum;
  uint4 rng;
  uint32_t mplan, midx, aplan, aidx, prev_opp;
  float prev_dist;
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
}

__device__ __forceinline__ uint64_t pack_fighter(const Fighter& f) {
  return (uint64_t)f.act | ((uint64_t)f.frame << 5) | ((uint64_t)f.stun << 14) | ((uint64_t)f.vital << 19) |
         ((uint64_t)f.guard << 21) | ((uint64_t)f.hits << 23) | ((uint64_t)f.buf << 25) |
         ((uint64_t)f.rsv << 30) | ((uint64_t)f.in_back << 35) | ((uint64_t)f.prox << 36) |
         ((uint64_t)f.won << 37) | ((uint64_t)f.hold << 38);
}

template <bool BOT>
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
  A.f0.hist = hist.x;
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
  if constexpr (BOT) {
    A.rng = s.rng[i];
    uint2 b = s.bot[i];
    A.mplan = b.x & 7;
    A.midx = (b.x >> 3) & 127;
    A.aplan = (b.x >> 10) & 7;
    A.aidx = (b.x >> 13) & 127;
    A.prev_opp = (b.x >> 20) & 31;
    A.prev_dist = __uint_as_float(b.y);
  }
}

template <bool BOT>
__device__ __forceinline__ void store_arena(const Arena& A, const DevState& s, int i) {
  uint64_t w0 = pack_fighter(A.f0), w1 = pack_fighter(A.f1);
  s.pos[i] = make_float2(A.f0.x, A.f1.x);
  s.hist[i] = make_uint2(A.f0.hist, A.f1.hist);
  s.fpk[i] = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
  uint32_t h = A.rec_count | (A.rec1 << 15) | (A.rec2 << 18) | (A.act1 << 21) | (A.act2 << 24) |
               ((uint32_t)A.pending << 27) | ((uint32_t)A.has_term << 28);
  s.aw[i] = make_int2(A.frame_count, (int)h);
  s.cum[i] = A.cum;
  if constexpr (BOT) {
    s.rng[i] = A.rng;
    s.bot[i] = make_uint2(A.mplan | (A.midx << 3) | (A.aplan << 10) | (A.aidx << 13) | (A.prev_opp << 20),
                          __float_as_uint(A.prev_dist));
  }
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
// basePosition.x + (dataRect.x * sign)   (TransformToFightRect, F:706-719)
template <int FM>
__device__ __forceinline__ float xform(float base, float rx, float sign) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return (float)__dadd_rn((double)base, __dmul_rn((double)rx, (double)sign));
  else return __fadd_rn(base, __fmul_rn(rx, sign));
}
// position.x += v * sign * Time.deltaTime   (F:300, 316)
template <int FM>
__device__ __forceinline__ float pos_plus_vel(float pos, float v, float sign) {
  if constexpr (FM == FS_FLOAT_DOUBLE)
    return (float)__dadd_rn((double)pos, __dmul_rn(__dmul_rn((double)v, (double)sign), (double)kDt));
  else return __fadd_rn(pos, __fmul_rn(__fmul_rn(v, sign), kDt));
}
// position.x -= v * sign * Time.deltaTime   (F:305)
template <int FM>
__device__ __forceinline__ float pos_minus_vel(float pos, float v, float sign) {
  if constexpr (FM == FS_FLOAT_DOUBLE)
    return (float)__dsub_rn((double)pos, __dmul_rn(__dmul_rn((double)v, (double)sign), (double)kDt));
  else return __fsub_rn(pos, __fmul_rn(__fmul_rn(v, sign), kDt));
}
// BoxBase.xMin / xMax (F:12-13): x is the centre
template <int FM>
__device__ __forceinline__ float bb_xmin(float x, float w) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return (float)__dsub_rn((double)x, (double)w / 2);
  else return __fsub_rn(x, w / 2.0f);
}
template <int FM>
__device__ __forceinline__ float bb_xmax(float x, float w) {
  if constexpr (FM == FS_FLOAT_DOUBLE) return (float)__dadd_rn((double)x, (double)w / 2);
  else return __fadd_rn(x, w / 2.0f);
}

// ---------------------------------------------------------------------------
// input (F:172-188, 569-666)
// ---------------------------------------------------------------------------
struct InputEval {
  bool fwd, back, special, atk_down, fdash, bdash;
};

// Left/Right -> (bit0 = backward, bit1 = forward).  P1 faces right, P2 left for
// the whole match (SetupBattleStart, F:124; BC:264-265).
__device__ __forceinline__ uint32_t rel_bits(uint32_t in, int k) {
  in &= 3;
  return k == 0 ? in : (((in & 1) << 1) | (in >> 1));
}
__device__ __forceinline__ uint32_t rel_hist(uint32_t h, int k) {
  return k == 0 ? h : (((h & 0x55555555u) << 1) | ((h >> 1) & 0x55555555u));
}
__device__ __forceinline__ uint32_t compact_even(uint32_t x) {
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0F0F0F0Fu;
  x = (x | (x >> 4)) & 0x00FF00FFu;
  x = (x | (x >> 8)) & 0x0000FFFFu;
  return x;
}

// UpdateInput + the reads UpdateActionRequest makes of the new history.
__device__ __forceinline__ InputEval update_input(Fighter& f, uint32_t in, int k) {
  const uint32_t old_hist = f.hist;
  const int old_hold = f.hold;
  const uint32_t in1 = (old_hist & 3) | (old_hold > 0 ? IN_ATTACK : 0);  // input[1] after the shift
  f.hist = (old_hist << 2) | (in & 3);
  f.hold = (in & IN_ATTACK) ? min(old_hold + 1, 63) : 0;
  InputEval e;
  const uint32_t r0 = rel_bits(in, k), r1 = rel_bits(in1, k);
  e.fwd = r0 & 2;
  e.back = r0 & 1;
  e.atk_down = (in & IN_ATTACK) && !(in1 & IN_ATTACK);                   // inputDown[0] & Attack
  e.special = !(in & IN_ATTACK) && old_hold >= kSpecialHoldFrame - 1;  // inputUp[0] & Attack, input[1..59] held
  // dash parsers over input[1..16] (bit j-1 of each mask = input[j])
  const uint32_t rh = rel_hist(old_hist, k);
  const uint32_t B = compact_even(rh), F = compact_even(rh >> 1), E = B | F;
  const uint32_t win = (1u << (kDashAllowFrame - 1)) - 1u;
  const uint32_t e8 = E & win;
  e.fdash = false;
  e.bdash = false;
  if (e8) {
    const int j = __builtin_ctz(e8);  // first i in 1..8 with any direction: i = j + 1
    const bool neutral = ((~E >> (j + 1)) & win) != 0;  // some input[i+1 .. i+8] with neither direction
    const bool isF = (F >> j) & 1, isB = (B >> j) & 1;
    e.fdash = (r0 & 2) && !(r1 & 2) && !isB && isF && neutral;
    e.bdash = (r0 & 1) && !(r1 & 1) && !isF && isB && neutral;
  }
  return e;
}

// ---------------------------------------------------------------------------
// action state machine (F:140-166, 201-286, 472-510, 546-563)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void set_action(Fighter& f, int a) {
  f.act = a;
  f.frame = 0;
  f.hits = 0;
  f.buf = NONE;
  f.rsv = NONE;
}

__device__ __forceinline__ void request_action(Fighter& f, int a) {
  const ActionInfo ai = sT.action[f.act];
  if (f.frame >= ai.frame_count) {
    set_action(f, a);
    return;
  }
  if (f.act == a) return;
  if (ai.always_cancel) {
    set_action(f, a);
    return;
  }
  const uint32_t row = sT.rows[ai.row + f.frame];
  if (sT.cancel[(row >> 21) & 15] & (1u << a)) f.buf = a;  // buffer or execute window lists `a`
}

__device__ __forceinline__ void increment_action_frame(Fighter& f) {
  if (f.stun > 0) {
    f.stun--;
    return;
  }
  f.frame++;
  const ActionInfo ai = sT.action[f.act];
  if (f.frame >= ai.frame_count && ai.loop_from >= 0) f.frame = ai.loop_from;
}

__device__ __forceinline__ void update_action_request(Fighter& f, const InputEval& e) {
  if (f.won) {
    request_action(f, A_WIN);
    return;
  }
  // reserved damage action, then buffered cancel (F:212-229).  Written as a value
  // select so the compiler cannot merge the two tails into a pointer phi (which
  // would pin the whole arena in scratch memory).
  const int rsv = f.rsv, buf = f.buf;
  const bool take_rsv = rsv != NONE && f.stun <= 0;
  const bool take_buf = !take_rsv && buf != NONE && (kCanCancelOnWhiff || f.hits > 0) && f.stun <= 0;
  if (take_rsv || take_buf) {
    set_action(f, take_rsv ? rsv : buf);
    return;
  }
  if (e.special) {
    request_action(f, (e.fwd || e.back) ? A_B_SPECIAL : A_N_SPECIAL);
  } else if (e.atk_down) {
    if ((f.act == A_N_ATTACK || f.act == A_B_ATTACK) && f.frame < sT.action[f.act].frame_count)
      request_action(f, A_N_SPECIAL);
    else
      request_action(f, (e.fwd || e.back) ? A_B_ATTACK : A_N_ATTACK);
  }
  if (e.fdash) request_action(f, A_DASH_FORWARD);
  else if (e.bdash) request_action(f, A_DASH_BACKWARD);
  f.in_back = e.back;
  if (e.fwd && e.back) request_action(f, A_STAND);
  else if (e.fwd) request_action(f, A_FORWARD);
  else if (e.back) request_action(f, f.prox ? A_GUARD_PROXIMITY : A_BACKWARD);
  else request_action(f, A_STAND);
  f.prox = false;
}

template <int FM>
__device__ __forceinline__ void update_movement(Fighter& f, float sign) {
  if (f.stun > 0) return;
  if (f.act == A_FORWARD) {
    f.x = pos_plus_vel<FM>(f.x, kForwardSpeed, sign);
  } else if (f.act == A_BACKWARD) {
    f.x = pos_minus_vel<FM>(f.x, kBackwardSpeed, sign);
  } else {
    const uint32_t vi = sT.rows[sT.action[f.act].row + f.frame] & 15;
    if (vi) {
      const float v = sT.vels[vi];
      if (v != 0.0f) f.x = pos_plus_vel<FM>(f.x, v, sign);
    }
  }
}

template <int FM>
__device__ __forceinline__ void update_boxes(Fighter& f, float sign) {
  const uint32_t row = sT.rows[sT.action[f.act].row + f.frame];
  f.push_rect = (row >> 4) & 31;
  f.hurtset = sT.hurtsets[(row >> 9) & 63];
  f.hitset = sT.hitsets[(row >> 15) & 63];
  f.px = xform<FM>(f.x, sT.rects[f.push_rect].x, sign);
  f.ux0 = xform<FM>(f.x, sT.rects[(f.hurtset >> 2) & 63].x, sign);
  f.ux1 = xform<FM>(f.x, sT.rects[(f.hurtset >> 8) & 63].x, sign);
  f.hx0 = xform<FM>(f.x, sT.rects[(f.hitset >> 2) & 63].x, sign);
  f.hx1 = xform<FM>(f.x, sT.rects[(f.hitset >> 11) & 63].x, sign);
}

// ApplyPositionChange (F:331-350): position and every box are shifted, not rebuilt
template <int FM>
__device__ __forceinline__ void apply_position_change(Fighter& f, float dx) {
  f.x = fadd<FM>(f.x, dx);
  f.px = fadd<FM>(f.px, dx);
  f.ux0 = fadd<FM>(f.ux0, dx);
  f.ux1 = fadd<FM>(f.ux1, dx);
  f.hx0 = fadd<FM>(f.hx0, dx);
  f.hx1 = fadd<FM>(f.hx1, dx);
}

// UpdatePushCharacterVsCharacter (BC:483-501) with UnityEngine.Rect semantics:
// x is xMin, xMax = width + x, Overlaps is strict.
template <int FM>
__device__ __forceinline__ void push_character_vs_character(Fighter& a, Fighter& b) {
  const float4 ra = sT.rects[a.push_rect], rb = sT.rects[b.push_rect];
  const float a_xmax = fadd<FM>(ra.z, a.px), b_xmax = fadd<FM>(rb.z, b.px);
  const float a_ymax = fadd<FM>(ra.w, ra.y), b_ymax = fadd<FM>(rb.w, rb.y);
  const bool overlap = b_xmax > a.px && b.px < a_xmax && b_ymax > ra.y && rb.y < a_ymax;
  if (!overlap) return;
  if (a.x < b.x) {
    float da, db;
    if constexpr (FM == FS_FLOAT_DOUBLE) {
      const double d = (double)a_xmax - (double)b.px;
      da = (float)(d * -1 / 2);
      db = (float)(d * 1 / 2);
    } else {
      const float d = __fsub_rn(a_xmax, b.px);
      da = d * -1.0f / 2.0f;
      db = d * 1.0f / 2.0f;
    }
    apply_position_change<FM>(a, da);
    apply_position_change<FM>(b, db);
  } else if (a.x > b.x) {
    float da, db;
    if constexpr (FM == FS_FLOAT_DOUBLE) {
      const double d = (double)b_xmax - (double)a.px;
      da = (float)(d * 1 / 2);
      db = (float)(d * -1 / 2);
    } else {
      const float d = __fsub_rn(b_xmax, a.px);
      da = d * 1.0f / 2.0f;
      db = d * -1.0f / 2.0f;
    }
    apply_position_change<FM>(a, da);
    apply_position_change<FM>(b, db);
  }
}

// UpdatePushCharacterVsBackground (BC:503-519) with BoxBase semantics
template <int FM>
__device__ __forceinline__ void push_character_vs_background(Fighter& f) {
  const float w = sT.rects[f.push_rect].z;
  const float xmin = bb_xmin<FM>(f.px, w);
  if (xmin < -kStageHalf) {
    apply_position_change<FM>(f, fsub<FM>(-kStageHalf, xmin));
  } else {
    const float xmax = bb_xmax<FM>(f.px, w);
    if (xmax > kStageHalf) apply_position_change<FM>(f, fsub<FM>(kStageHalf, xmax));
  }
}

// BoxBase.Overlaps (F:17-25), inclusive; `self` is the hitbox, `other` the hurtbox
template <int FM>
__device__ __forceinline__ bool box_overlaps(float sx, float4 sr, float ox, float4 orr) {
  const bool c1 = bb_xmax<FM>(ox, orr.z) >= bb_xmin<FM>(sx, sr.z);
  const bool c2 = bb_xmin<FM>(ox, orr.z) <= bb_xmax<FM>(sx, sr.z);
  const bool c3 = fadd<FM>(orr.y, orr.w) >= sr.y;
  const bool c4 = orr.y <= fadd<FM>(sr.y, sr.w);
  return c1 && c2 && c3 && c4;
}

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
  if (f.act == A_BACKWARD || sT.action[f.act].guard_type) {
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

// one attacker of UpdateHitboxHurtboxCollision (BC:521-591)
template <int FM>
__device__ __forceinline__ void collide(Fighter& att, Fighter& def) {
  const int nh = att.hitset & 3;
  if (nh == 0) return;  // only attack actions carry hitboxes
  const int nu = def.hurtset & 3;
  bool hit = false, prox = false;
  int atk = 0;
  for (int h = 0; h < nh; h++) {
    const uint32_t hb = (att.hitset >> (2 + 9 * h)) & 511;
    const int aidx = (hb >> 6) & 3;
    if (att.hits >= sT.attacks[aidx].number_of_hit) continue;  // CanAttackHit (F:408-420)
    const float4 hr = sT.rects[hb & 63];
    const float hx = h == 0 ? att.hx0 : att.hx1;
    for (int u = 0; u < nu; u++) {
      const float4 ur = sT.rects[(def.hurtset >> (2 + 6 * u)) & 63];
      const float ux = u == 0 ? def.ux0 : def.ux1;
      if (box_overlaps<FM>(hx, hr, ux, ur)) {
        if ((hb >> 8) & 1) {
          prox = true;
        } else {
          hit = true;
          atk = aidx;
          break;
        }
      }
    }
    if (hit) break;
  }
  if (hit) {
    att.hits++;  // NotifyAttackHit (F:352-355)
    const AttackInfo ad = sT.attacks[atk];
    const int res = notify_damaged(def, ad);
    const int stun = res == DR_GUARD ? ad.guard_stun : res == DR_GUARD_BREAK ? ad.guard_break_stun : ad.hit_stun;
    att.stun = stun;  // SetHitStun on both (BC:576-578)
    def.stun = stun;
  } else if (prox) {
    if (def.in_back) def.prox = true;  // NotifyInProximityGuardRange (F:400-406)
  }
}

// ---------------------------------------------------------------------------
// bot: BattleAI for P2 (AI:10-403) with queues as (plan, index)
// ---------------------------------------------------------------------------
enum { MP_NEUTRAL, MP_FAR1, MP_FAR2, MP_MID1, MP_MID2, MP_FALLBACK1, MP_FALLBACK2 };
enum { AP_NONE, AP_ONE_HIT, AP_TWO_HIT, AP_IMMEDIATE_SPECIAL, AP_DELAY_SPECIAL };
__device__ __forceinline__ uint32_t move_plan_len(uint32_t plan) {  // AI:192-253
  return plan == MP_FAR1 ? 90u : plan == MP_FAR2 ? 56u : plan == MP_MID1 ? 70u : plan == MP_MID2 ? 33u
       : plan == MP_FALLBACK1 ? 60u : plan == MP_FALLBACK2 ? 63u : 30u;
}
__device__ __forceinline__ uint32_t attack_plan_len(uint32_t plan) {  // AI:255-312
  return plan == AP_ONE_HIT ? 19u : plan == AP_TWO_HIT ? 23u : plan == AP_IMMEDIATE_SPECIAL ? 61u
       : plan == AP_DELAY_SPECIAL ? 121u : 30u;
}

__device__ __forceinline__ uint32_t rng_next(uint4& s) {  // UnityEngine.Random Xorshift128
  const uint32_t t = s.x ^ (s.x << 11);
  s.x = s.y;
  s.y = s.z;
  s.z = s.w;
  s.w = s.w ^ (s.w >> 19) ^ t ^ (t >> 8);
  return s.w;
}
__device__ __forceinline__ int rng_range(uint4& s, int mn, int mx) {  // Random.Range(int, int)
  return mn + (int)(rng_next(s) % (uint32_t)(mx - mn));
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
__device__ __forceinline__ uint32_t move_plan_input(uint32_t plan, uint32_t i) {
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
__device__ __forceinline__ uint32_t attack_plan_input(uint32_t plan, uint32_t i) {
  switch (plan) {
    case AP_ONE_HIT: return i == 0 ? IN_ATTACK : 0u;
    case AP_TWO_HIT: return (i == 0 || i == 4) ? IN_ATTACK : 0u;
    case AP_IMMEDIATE_SPECIAL: return i < 60 ? IN_ATTACK : 0u;
    case AP_DELAY_SPECIAL: return i < 120 ? IN_ATTACK : 0u;
    default: return 0u;
  }
}

__device__ __forceinline__ uint32_t select_movement(uint4& rng, float d) {  // AI:68-126
  if (d > 4.0f) return rng_range(rng, 0, 2) == 0 ? MP_FAR1 : MP_FAR2;
  if (d > 3.0f) {
    const int r = rng_range(rng, 0, 7);
    return r <= 1 ? MP_MID1 : r <= 3 ? MP_MID2 : r == 4 ? MP_FAR1 : r == 5 ? MP_FAR2 : MP_NEUTRAL;
  }
  if (d > 2.5f) {
    const int r = rng_range(rng, 0, 5);
    return r == 0 ? MP_MID1 : r == 1 ? MP_MID2 : r == 2 ? MP_FALLBACK1 : r == 3 ? MP_FALLBACK2 : MP_NEUTRAL;
  }
  if (d > 2.0f) {
    const int r = rng_range(rng, 0, 4);
    return r == 0 ? MP_FALLBACK1 : r == 1 ? MP_FALLBACK2 : MP_NEUTRAL;
  }
  const int r = rng_range(rng, 0, 3);
  return r == 0 ? MP_FALLBACK1 : r == 1 ? MP_FALLBACK2 : MP_NEUTRAL;
}

__device__ __forceinline__ uint32_t select_attack(uint4& rng, float d, uint32_t opp) {  // AI:128-190
  if (opp == A_DAMAGE || opp == A_GUARD_BREAK || opp == A_N_SPECIAL || opp == A_B_SPECIAL) return AP_TWO_HIT;
  if (d > 4.0f) return rng_range(rng, 0, 4) <= 3 ? AP_NONE : AP_DELAY_SPECIAL;
  if (d > 3.0f) {
    if (opp == A_N_ATTACK || opp == A_B_ATTACK) return AP_TWO_HIT;
    const int r = rng_range(rng, 0, 5);
    return r <= 1 ? AP_NONE : r <= 3 ? AP_ONE_HIT : AP_DELAY_SPECIAL;
  }
  if (d > 2.5f) {
    const int r = rng_range(rng, 0, 3);
    return r == 0 ? AP_NONE : r == 1 ? AP_ONE_HIT : AP_TWO_HIT;
  }
  if (d > 2.0f) {
    const int r = rng_range(rng, 0, 6);
    return r <= 1 ? AP_ONE_HIT : r <= 3 ? AP_TWO_HIT : r == 4 ? AP_IMMEDIATE_SPECIAL : AP_DELAY_SPECIAL;
  }
  return rng_range(rng, 0, 3) == 0 ? AP_ONE_HIT : AP_TWO_HIT;
}

template <int FM>
__device__ __forceinline__ float bot_distance(const Arena& A) {  // Mathf.Abs(f2.x - f1.x) (AI:370-373)
  return fabsf(fsub<FM>(A.f1.x, A.f0.x));
}

template <int FM>
__device__ __forceinline__ void bot_reset(Arena& A) {  // AI:393-403
  A.mplan = A.midx = A.aplan = A.aidx = 0;
  A.prev_dist = bot_distance<FM>(A);
  A.prev_opp = A.f0.act;
}

// getNextAIInput (AI:41-66).  The ascending copy loop of UpdateFightState
// (AI:358-361) makes fightStates[5] the *previous* call's state.
template <int FM>
__device__ __forceinline__ uint32_t bot_next_input(Arena& A) {
  const float d = A.prev_dist;
  const uint32_t opp = A.prev_opp;
  A.prev_dist = bot_distance<FM>(A);
  A.prev_opp = A.f0.act;
  uint32_t input = 0;
  if (A.mplan) {
    input |= move_plan_input(A.mplan - 1, A.midx);
    if (++A.midx == move_plan_len(A.mplan - 1)) A.mplan = 0;
  } else {
    A.mplan = select_movement(A.rng, d) + 1;
    A.midx = 0;
  }
  if (A.aplan) {
    input |= attack_plan_input(A.aplan - 1, A.aidx);
    if (++A.aidx == attack_plan_len(A.aplan - 1)) A.aplan = 0;
  } else {
    A.aplan = select_attack(A.rng, d, opp) + 1;
    A.aidx = 0;
  }
  return input;
}

// ---------------------------------------------------------------------------
// round flow (BC:138-345)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void record_input(Arena& A, uint32_t p1, uint32_t p2) {  // BC:593-607
  if (A.rec_count >= kMaxRecording) return;
  A.rec1 = p1;
  A.rec2 = p2;
  A.rec_count++;
}

template <int FM>
__device__ __forceinline__ void physics_tail(Arena& A) {  // movement, boxes, pushes (shared by all tick kinds)
  update_movement<FM>(A.f0, 1.0f);
  update_movement<FM>(A.f1, -1.0f);
  update_boxes<FM>(A.f0, 1.0f);
  update_boxes<FM>(A.f1, -1.0f);
  push_character_vs_character<FM>(A.f0, A.f1);
  push_character_vs_background<FM>(A.f0);
  push_character_vs_background<FM>(A.f1);
}

// UpdateFightState (BC:347-364); returns battleOver (BC:212-213)
template <int FM>
__device__ __forceinline__ bool fight_tick(Arena& A) {
  A.frame_count++;
  record_input(A, A.act1, A.act2);
  const InputEval e0 = update_input(A.f0, A.act1, 0);
  const InputEval e1 = update_input(A.f1, A.act2, 1);
  increment_action_frame(A.f0);
  increment_action_frame(A.f1);
  update_action_request(A.f0, e0);
  update_action_request(A.f1, e1);
  physics_tail<FM>(A);
  collide<FM>(A.f0, A.f1);
  collide<FM>(A.f1, A.f0);
  return A.f0.vital <= 0 || A.f1.vital <= 0;
}

__device__ __forceinline__ void ko_clear_input(Arena& A) {  // ChangeRoundState(KO): ClearInput (BC:292-299)
  A.f0.hist = A.f1.hist = 0;
  A.f0.hold = A.f1.hold = 0;
}

__device__ __forceinline__ void setup_battle_start(Fighter& f, float x) {  // F:120-135
  f.x = x;
  f.vital = 1;
  f.guard = kStartGuard;
  f.won = false;
  f.hist = 0;
  f.hold = 0;
  set_action(f, A_STAND);
}

// KO tick -> End (winner), End tick (BC:221-243, 306-325, 371-381), reduced to
// its observable effects.  The End tick runs IncrementActionFrame,
// UpdateActionRequest, movement, boxes and pushes, but SetupBattleStart (next
// tick) overwrites position, action, frame, hit count, buffer, reserve, vital,
// guard, hasWon and the input history.  What survives is (a) the hitstun
// decrement and (b) UpdateActionRequest clearing isInputBackward /
// isReserveProximityGuard -- which it does unless it returned early: for the
// winner (hasWon), or on the reserve / buffer paths (F:204-229).  The input
// history was cleared at KO, so the fall-through path sees no input.
__device__ __forceinline__ void end_tick_effects(Fighter& f, bool won) {
  const bool stunned = f.stun > 0;
  f.stun -= stunned ? 1 : 0;  // IncrementActionFrame (F:150-154); the frame itself is overwritten
  const bool early = won || (f.rsv != NONE && f.stun <= 0) ||
                     (f.buf != NONE && (kCanCancelOnWhiff || f.hits > 0) && f.stun <= 0);
  f.in_back = early ? f.in_back : false;
  f.prox = early ? f.prox : false;
}

__device__ __forceinline__ void ko_and_end_ticks(Arena& A) {
  const bool d0 = A.f0.vital <= 0, d1 = A.f1.vital <= 0;
  end_tick_effects(A.f0, A.f0.won || (d1 && !d0));  // a sole survivor gets RequestWinAction (BC:310-323)
  end_tick_effects(A.f1, A.f1.won || (d0 && !d1));
}

// Intro tick for one fighter right after SetupBattleStart (BC:329-345): the stale
// actor input enters the cleared history, the frame advances unless in hitstun,
// and RequestAction(STAND) on STAND is a no-op.  Movement, boxes and both pushes
// are no-ops here: STAND has no movement window, and base pushboxes at x = -2 / +2
// neither overlap each other nor the stage edges.
__device__ __forceinline__ void intro_tick_fighter(Fighter& f, uint32_t in) {
  f.hist = in & 3;
  f.hold = (in & IN_ATTACK) ? 1 : 0;
  const bool stunned = f.stun > 0;
  f.stun -= stunned ? 1 : 0;
  f.frame = stunned ? 0 : 1;
}

// Stop tick -> Intro (SetupBattleStart, bot Reset), Intro tick with the stale
// actor inputs, -> Fight (frameCount = -1) and the state(-1) emission with the
// bot's request (BC:178-200, 262-291, 329-345)
template <int FM, bool BOT>
__device__ __forceinline__ void stop_intro_fight(Arena& A) {
  setup_battle_start(A.f0, kP1StartX);
  setup_battle_start(A.f1, kP2StartX);
  if constexpr (BOT) bot_reset<FM>(A);
  record_input(A, A.act1, A.act2);
  intro_tick_fighter(A.f0, A.act1);
  intro_tick_fighter(A.f1, A.act2);
  A.frame_count = -1;
  A.rec_count = 0;
  if constexpr (BOT) A.act2 = bot_next_input<FM>(A);
}

// ---------------------------------------------------------------------------
// outputs (FE:336-380, 537-549)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void write_obs(const Arena& A, uint8_t* guard, uint8_t* move, float* move_frame,
                                          float* position, int32_t* frame, uint8_t* action, uint8_t* hitstun,
                                          size_t r) {
  int a0 = A.f0.act, a1 = A.f1.act;
  if (a0 == A_DEAD || a0 == A_WIN) a0 = A_STAND;  // FE:537-549
  if (a1 == A_DEAD || a1 == A_WIN) a1 = A_STAND;
  const int m[2] = {a0, a1};
  const int mf[2] = {(a0 == A_STAND || a0 == A_FORWARD || a0 == A_BACKWARD) ? 0 : A.f0.frame,  // FE:339-358
                     (a1 == A_STAND || a1 == A_FORWARD || a1 == A_BACKWARD) ? 0 : A.f1.frame};
  const bool rec = A.rec_count > 0;
  reinterpret_cast<uchar2*>(guard)[r] = make_uchar2((uint8_t)A.f0.guard, (uint8_t)A.f1.guard);
  reinterpret_cast<uchar2*>(move)[r] = make_uchar2((uint8_t)m[0], (uint8_t)m[1]);
  reinterpret_cast<float2*>(move_frame)[r] = make_float2((float)mf[0], (float)mf[1]);
  reinterpret_cast<float2*>(position)[r] = make_float2(A.f0.x, A.f1.x);
  frame[r] = A.frame_count;
  reinterpret_cast<uchar2*>(action)[r] = make_uchar2(rec ? (uint8_t)A.rec1 : 0, rec ? (uint8_t)A.rec2 : 0);
  reinterpret_cast<uchar2*>(hitstun)[r] = make_uchar2((uint8_t)A.f0.stun, (uint8_t)A.f1.stun);
}

__device__ __forceinline__ void write_main(const Arena& A, const DevOutputs& o, size_t r) {
  write_obs(A, o.guard, o.move, o.move_frame, o.position, o.frame, o.action, o.hitstun, r);
}
__device__ __forceinline__ void write_final(const Arena& A, const DevOutputs& o, size_t r) {
  write_obs(A, o.final_guard, o.final_move, o.final_move_frame, o.final_position, o.final_frame, o.final_action,
            o.final_hitstun, r);
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
// one env-step of one arena: FootsiesEnv.step (FE:518-570) over the synced game
// ---------------------------------------------------------------------------
template <int FM, int P2>
__device__ __forceinline__ void env_step(Arena& A, uint32_t a1, uint32_t a2, const StepParams& p, size_t r) {
  constexpr bool BOT = P2 == FS_P2_BOT;
  const DevOutputs& o = p.out;
  if (A.pending) {  // FS_AUTORESET_NEXT_STEP: this step runs the reset burst only
    ko_and_end_ticks(A);
    stop_intro_fight<FM, BOT>(A);
    A.pending = false;
    A.has_term = false;
    A.cum = 0.0;
    write_main(A, o, r);
    o.reward[r] = 0.0;
    o.terminated[r] = 0;
    o.truncated[r] = 0;
    return;
  }
  A.act1 = a1;
  if constexpr (P2 == FS_P2_EXTERNAL) A.act2 = a2;
  else if constexpr (P2 == FS_P2_NOOP) A.act2 = 0;
  const int g1 = A.f0.guard, g2 = A.f1.guard;  // guards of FE._current_state
  const bool over = fight_tick<FM>(A);
  double reward;
  if (p.dense_reward) {  // FE:388-405
    reward = 0.0;
    if (A.f0.guard < g1) reward -= 0.3;
    if (A.f1.guard < g2) reward += 0.3;
    A.cum += reward;
    if (over) reward += (double)(A.f1.vital == 0 ? 1 : -1) - A.cum;
  } else {  // FE:382-386
    reward = over ? (A.f1.vital == 0 ? 1.0 : -1.0) : 0.0;
  }
  if (over) {
    ko_clear_input(A);
    if (p.autoreset_mode == FS_AUTORESET_SAME_STEP) {
      write_final(A, o, r);
      ko_and_end_ticks(A);
      stop_intro_fight<FM, BOT>(A);
      A.cum = 0.0;
      A.has_term = false;
    } else {
      A.pending = true;
      A.has_term = true;
    }
  } else {
    if constexpr (BOT) A.act2 = bot_next_input<FM>(A);  // TrainingManager.Step -> RequestNextInput
    A.has_term = false;
  }
  write_main(A, o, r);
  o.reward[r] = reward;
  o.terminated[r] = over ? 1 : 0;
  o.truncated[r] = 0;
}

template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step(StepParams p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  stage_tables();
  if (i >= p.n_envs) return;
  constexpr bool BOT = P2 == FS_P2_BOT;
  Arena A;
  load_arena<BOT>(A, p.st, i);
  for (int k = 0; k < p.n_steps; k++) {
    const size_t arow = (size_t)k * p.n_envs + i;
    const size_t orow = (size_t)k * p.out_stride_steps * p.n_envs + i;
    const uint64_t t = p.t0 + (uint64_t)k;
    const uint32_t a1 = p.p1 ? p.p1[arow] : hash_action(p.action_seed, i, t, 0);
    uint32_t a2 = 0;
    if constexpr (P2 == FS_P2_EXTERNAL) a2 = p.p2 ? p.p2[arow] : hash_action(p.action_seed, i, t, 1);
    env_step<FM, P2>(A, a1 & 7u, a2 & 7u, p, orow);
  }
  store_arena<BOT>(A, p.st, i);
}

// FootsiesEnv.reset (FE:482-515) / RESET (BC:143-146) / game start (BC:105-128)
template <int FM, int P2>
__global__ __launch_bounds__(256) void k_reset(ResetParams p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  stage_tables();
  if (i >= p.n_envs) return;
  if (!p.init && p.mask && !p.mask[i]) return;
  constexpr bool BOT = P2 == FS_P2_BOT;
  Arena A;
  if (p.init) {  // `new Fighter()` defaults (F:73-112), round state Stop
    for (int k = 0; k < 2; k++) {
      Fighter& f = k == 0 ? A.f0 : A.f1;
      f.x = 0.0f;
      f.hist = 0;
      f.act = A_STAND;
      f.frame = f.stun = f.vital = f.guard = f.hits = f.hold = 0;
      f.buf = f.rsv = NONE;
      f.in_back = f.prox = f.won = false;
    }
    A.frame_count = 0;
    A.rec_count = A.rec1 = A.rec2 = A.act1 = A.act2 = 0;
    A.pending = false;
    A.has_term = true;
    A.cum = 0.0;
    A.rng = rng_init((int32_t)(uint32_t)(p.base_seed + (uint64_t)i));
    A.mplan = A.midx = A.aplan = A.aidx = A.prev_opp = 0;
    A.prev_dist = 0.0f;
  } else {
    load_arena<BOT>(A, p.st, i);
  }
  if (p.seeds) A.rng = rng_init((int32_t)(uint32_t)p.seeds[i]);  // SEED (BC:170-173)
  const bool hard = p.init || p.flags == FS_RESET_HARD || !A.has_term;
  if (A.pending) {  // finish the burst Unity ran after the terminal frame
    ko_and_end_ticks(A);
    stop_intro_fight<FM, BOT>(A);
    A.pending = false;
  }
  if (hard) stop_intro_fight<FM, BOT>(A);
  A.cum = 0.0;
  A.has_term = p.init ? true : false;
  write_main(A, p.out, i);
  p.out.reward[i] = 0.0;
  p.out.terminated[i] = 0;
  p.out.truncated[i] = 0;
  store_arena<BOT>(A, p.st, i);
}

// synthetic action stream (fs_hash_actions), one thread per (step, arena)
__global__ __launch_bounds__(256) void k_hash_actions(int n_envs, int n_steps, uint64_t seed, uint64_t t0,
                                                       uint8_t* p1, uint8_t* p2) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)n_envs * n_steps) return;
  const uint64_t env = idx % (size_t)n_envs, k = idx / (size_t)n_envs;
  p1[idx] = (uint8_t)hash_action(seed, env, t0 + k, 0);
  if (p2) p2[idx] = (uint8_t)hash_action(seed, env, t0 + k, 1);
}

// canonical export (fs_get_state / fs_get_env_state)
template <bool BOT>
__global__ __launch_bounds__(256) void k_get_state(DevState st, fs_arena_state* dst, fs_env_state* env, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Arena A;
  load_arena<BOT>(A, st, i);
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
      g.input_dir_history = f.hist;
      g.attack_hold = f.hold;
      g.is_input_backward = f.in_back;
      g.is_reserve_proximity_guard = f.prox;
      g.has_won = f.won;
      g.pad0 = 0;
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
    if constexpr (BOT) {
      s.rng[0] = A.rng.x;
      s.rng[1] = A.rng.y;
      s.rng[2] = A.rng.z;
      s.rng[3] = A.rng.w;
      s.move_plan = A.mplan ? (int32_t)A.mplan - 1 : -1;
      s.move_index = A.mplan ? (int32_t)A.midx : 0;
      s.attack_plan = A.aplan ? (int32_t)A.aplan - 1 : -1;
      s.attack_index = A.aplan ? (int32_t)A.aidx : 0;
      s.prev_distance = A.prev_dist;
      s.prev_opponent_action = kActionId[A.prev_opp];
    } else {
      s.rng[0] = s.rng[1] = s.rng[2] = s.rng[3] = 0;
      s.move_plan = s.attack_plan = -1;
      s.move_index = s.attack_index = 0;
      s.prev_distance = 0.0f;
      s.prev_opponent_action = 0;
    }
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

template <bool BOT>
__global__ __launch_bounds__(256) void k_set_state(DevState st, const fs_arena_state* src, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fs_arena_state s = src[i];
  Arena A;
  for (int k = 0; k < 2; k++) {
    const fs_fighter_state& g = s.f[k];
    Fighter& f = k == 0 ? A.f0 : A.f1;
    f.x = g.position_x;
    f.act = action_index_of(g.action_id);
    f.frame = g.action_frame;
    f.hits = g.hit_count;
    f.stun = g.hitstun;
    f.vital = g.vital;
    f.guard = g.guard;
    f.buf = g.buffer_action_id < 0 ? NONE : action_index_of(g.buffer_action_id);
    f.rsv = g.reserve_action_id < 0 ? NONE : action_index_of(g.reserve_action_id);
    f.hist = g.input_dir_history;
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
  if constexpr (BOT) {
    A.rng = make_uint4(s.rng[0], s.rng[1], s.rng[2], s.rng[3]);
    A.mplan = s.move_plan < 0 ? 0u : (uint32_t)s.move_plan + 1;
    A.midx = s.move_plan < 0 ? 0u : (uint32_t)s.move_index;
    A.aplan = s.attack_plan < 0 ? 0u : (uint32_t)s.attack_plan + 1;
    A.aidx = s.attack_plan < 0 ? 0u : (uint32_t)s.attack_index;
    A.prev_dist = s.prev_distance;
    A.prev_opp = (uint32_t)action_index_of(s.prev_opponent_action);
  }
  store_arena<BOT>(A, st, i);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
constexpr int kBlock = 256;
static inline dim3 grid_for(int n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

template <int FM>
static hipError_t launch_step_fm(const StepParams& p, int p2_mode, hipStream_t s) {
  switch (p2_mode) {
    case FS_P2_EXTERNAL: hipLaunchKernelGGL((k_step<FM, FS_P2_EXTERNAL>), grid_for(p.n_envs), dim3(kBlock), 0, s, p); break;
    case FS_P2_BOT: hipLaunchKernelGGL((k_step<FM, FS_P2_BOT>), grid_for(p.n_envs), dim3(kBlock), 0, s, p); break;
    default: hipLaunchKernelGGL((k_step<FM, FS_P2_NOOP>), grid_for(p.n_envs), dim3(kBlock), 0, s, p); break;
  }
  return hipGetLastError();
}

hipError_t launch_step(const StepParams& p, int float_mode, int p2_mode, hipStream_t s) {
  return float_mode == FS_FLOAT_DOUBLE ? launch_step_fm<FS_FLOAT_DOUBLE>(p, p2_mode, s)
                                       : launch_step_fm<FS_FLOAT_STRICT32>(p, p2_mode, s);
}

template <int FM>
static hipError_t launch_reset_fm(const ResetParams& p, int p2_mode, hipStream_t s) {
  switch (p2_mode) {
    case FS_P2_EXTERNAL: hipLaunchKernelGGL((k_reset<FM, FS_P2_EXTERNAL>), grid_for(p.n_envs), dim3(kBlock), 0, s, p); break;
    case FS_P2_BOT: hipLaunchKernelGGL((k_reset<FM, FS_P2_BOT>), grid_for(p.n_envs), dim3(kBlock), 0, s, p); break;
    default: hipLaunchKernelGGL((k_reset<FM, FS_P2_NOOP>), grid_for(p.n_envs), dim3(kBlock), 0, s, p); break;
  }
  return hipGetLastError();
}

hipError_t launch_reset(const ResetParams& p, int float_mode, int p2_mode, hipStream_t s) {
  return float_mode == FS_FLOAT_DOUBLE ? launch_reset_fm<FS_FLOAT_DOUBLE>(p, p2_mode, s)
                                       : launch_reset_fm<FS_FLOAT_STRICT32>(p, p2_mode, s);
}

hipError_t launch_hash_actions(int n_envs, int n_steps, uint64_t seed, uint64_t t0, uint8_t* p1, uint8_t* p2,
                               hipStream_t s) {
  const size_t total = (size_t)n_envs * n_steps;
  hipLaunchKernelGGL(k_hash_actions, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n_envs,
                     n_steps, seed, t0, p1, p2);
  return hipGetLastError();
}

hipError_t launch_get_state(const DevState& st, fs_arena_state* dst, fs_env_state* env, int n, int p2_mode,
                            hipStream_t s) {
  if (p2_mode == FS_P2_BOT) hipLaunchKernelGGL(k_get_state<true>, grid_for(n), dim3(kBlock), 0, s, st, dst, env, n);
  else hipLaunchKernelGGL(k_get_state<false>, grid_for(n), dim3(kBlock), 0, s, st, dst, env, n);
  return hipGetLastError();
}

hipError_t launch_set_state(const DevState& st, const fs_arena_state* src, int n, int p2_mode, hipStream_t s) {
  if (p2_mode == FS_P2_BOT) hipLaunchKernelGGL(k_set_state<true>, grid_for(n), dim3(kBlock), 0, s, st, src, n);
  else hipLaunchKernelGGL(k_set_state<false>, grid_for(n), dim3(kBlock), 0, s, st, src, n);
  return hipGetLastError();
}

}  // namespace fsk
