// fs_arena1.h -- the fused rollout kernel with ONE lane per arena (included by fs_kernels.hip,
// inside namespace fsk, after the two-lane code whose per-fighter functions it reuses).
//
// The two-lane kernel (lane 2a+k = fighter k of arena a) issues every instruction of a tick for
// 32 arenas per wave; the arena-level work (frame count, recording, KO test, the f64 reward, the
// per-arena stores and the reset burst) runs as identical replicas on both lanes, and the pair
// phases (pushes, collision, KO) cross the pair with DPP moves.  Here one lane runs a whole
// arena: the per-fighter phases run twice per lane (the compiler interleaves the two independent
// chains, so one wave has two LDS round trips in flight where the two-lane wave had one), the
// arena-level work once, the pair phases without exchanges, and a lane stores both fighters'
// values of a [N][2] output as one 2- or 8-byte store.  A wave then covers 64 arenas, so C3's
// 65 536 arenas run one wave per SIMD.
//
// Semantics are exactly env_step's (fs_kernels.hip), phase by phase and in the same operation
// order; the CPU oracle and the GPU parity suite hold both kernels to the same bits.  Used for
// the fused launches with action rows (fs_step_n, and fs_step_n_packed: k_step_n1_packed) and a
// remote, idle or bot P2; the one-tick, hashed-action, policy and per-arena-actor launches keep
// the two-lane kernel.
//
// Paths: BC = Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs, AI = Assets/Script/BattleAI.cs,
// FE = footsies-gym/footsies_gym/envs/footsies.py.

// P2's whole BattleAI on the arena's lane (the two-lane kernel splits its queues over the pair)
struct Bot1 {
  uint4 rng;                          // the game's UnityEngine.Random
  uint32_t mplan, midx, aplan, aidx;  // plans stored + 1 (0 = empty queue), dequeued counts
  uint32_t prev_opp;                  // fightStates[5]: opponent action idx ...
  float prev_dist;                    // ... and distance
};

// The bot tables one call reads, issued at the top of the tick from the state before the call
struct BotPre1 {
  uint32_t mcode, acode;  // codes[q][plan][idx >> 4] of the movement / attack queue
  uint32_t mlen, alen;    // len[q][plan]
  BotDraw mw, aw;         // draw[q][bucket of the previous distance]
};

__device__ __forceinline__ BotPre1 bot_prefetch1(const Bot1& b) {
  const BotTables& T = bots<false>();
  const uint32_t mp = b.mplan != 0 ? b.mplan - 1 : 0u, ap = b.aplan != 0 ? b.aplan - 1 : 0u;
  const uint32_t bk = bot_bucket(b.prev_dist);
  BotPre1 r;
  r.mcode = T.codes[1][mp][b.midx >> 4];
  r.acode = T.codes[0][ap][b.aidx >> 4];
  r.mlen = T.len[1][mp];
  r.alen = T.len[0][ap];
  r.mw = T.draw[1][bk];
  r.aw = T.draw[0][bk];
  return r;
}

// getNextAIInput (AI:41-66) with both queues on one lane, branch-free: the movement queue is
// dequeued or refilled by a draw, then the attack queue; the RNG advances by the draws taken,
// movement first (the order of SelectMovement / SelectAttack).  Same state transitions as
// bot_next_input's lane pair.
__device__ __forceinline__ uint32_t bot_next_input1(Bot1& b, float dist, uint32_t opp_act, const BotPre1& pre) {
  const float d = b.prev_dist;
  const uint32_t opp = b.prev_opp;
  b.prev_dist = dist;
  b.prev_opp = opp_act;
  const uint32_t bucket = bot_bucket(d);
  const bool mbusy = b.mplan != 0, abusy = b.aplan != 0;
  const uint32_t mi = b.midx, ai = b.aidx;
  const uint32_t min_ = mbusy ? (pre.mcode >> (2 * (mi & 15))) & 3u : 0u;            // Left / Right bits
  const uint32_t ain = abusy ? ((pre.acode >> (2 * (ai & 15))) & 3u) << 2 : 0u;       // IN_ATTACK
  const bool forced = attack_forced(bucket, opp);
  const bool dm = !mbusy, da = !abusy & !forced;
  uint4 s1 = b.rng;
  const uint32_t x1 = rng_next(s1);
  uint4 s2 = s1;
  const uint32_t x2 = rng_next(s2);
  const uint4 s0 = b.rng;
  b.rng = sel4(dm & da, s2, sel4(dm | da, s1, s0));
  const uint32_t newm = (pre.mw.map >> (4 * draw_mod(x1, pre.mw))) & 15u;
  const uint32_t drawn_a = (pre.aw.map >> (4 * draw_mod(dm ? x2 : x1, pre.aw))) & 15u;
  const uint32_t newa = forced ? (uint32_t)AP_TWO_HIT : drawn_a;
  const uint32_t mi1 = mi + 1, ai1 = ai + 1;
  b.mplan = mbusy ? (mi1 == pre.mlen ? 0u : b.mplan) : newm + 1;
  b.midx = mbusy ? mi1 : 0u;
  b.aplan = abusy ? (ai1 == pre.alen ? 0u : b.aplan) : newa + 1;
  b.aidx = abusy ? ai1 : 0u;
  return min_ | ain;
}

struct Arena1 {
  Fighter f0, f1;
  int frame_count;
  uint32_t rec_count;
  uint32_t rec0, rec1;    // recordingP1/P2Input[index - 1]
  uint32_t act0, act1;    // the remote actors' inputs (TrainingRemoteActor.input)
  uint32_t bin;           // P2 bot's input (TrainingBattleAIActor.input), bot handles
  uint32_t pending, has_term;
  double cum;
  AInfo ai0, ai1;         // ActionInfo of each fighter's action (re-read at the end of every tick)
  Bot1 bot;               // FS_P2_BOT only
};

template <int V>
__device__ __forceinline__ void load_arena1(Arena1& A, const DevState& s, int a) {
  const float2 pos = s.pos[a];
  const uint2 hist = s.hist[a];
  const uint4 pk = s.fpk[a];
  const int2 aw = s.aw[a];
  A.cum = s.cum[a];
  unpack_fighter(A.f0, pk.x, pk.y);
  unpack_fighter(A.f1, pk.z, pk.w);
  A.f0.x = pos.x;
  A.f1.x = pos.y;
  A.f0.hist = hist.x;
  A.f1.hist = hist.y;
  const uint32_t h = (uint32_t)aw.y;
  A.frame_count = aw.x;
  A.rec_count = h & 0x7fff;
  A.rec0 = (h >> 15) & 7;
  A.rec1 = (h >> 18) & 7;
  A.act0 = (h >> 21) & 7;
  A.act1 = (h >> 24) & 7;
  A.pending = (h >> 27) & 1;
  A.has_term = (h >> 28) & 1;
  A.bin = 0;
  if constexpr (V == FS_P2_BOT) {
    A.bot.rng = s.rng[a];
    const uint2 b = s.bot[a];
    A.bot.mplan = b.x & 7;
    A.bot.midx = (b.x >> 3) & 127;
    A.bot.aplan = (b.x >> 10) & 7;
    A.bot.aidx = (b.x >> 13) & 127;
    A.bot.prev_opp = (b.x >> 20) & 31;
    A.bot.prev_dist = __uint_as_float(b.y);
    A.bin = (b.x >> 26) & 7;  // (a bot-created P2 is Reset at every Intro: always ready)
  }
}

template <int V>
__device__ __forceinline__ void store_arena1(const Arena1& A, const DevState& s, int a) {
  const uint64_t w0 = pack_fighter(A.f0), w1 = pack_fighter(A.f1);
  s.pos[a] = make_float2(A.f0.x, A.f1.x);
  s.hist[a] = make_uint2(A.f0.hist, A.f1.hist);
  s.fpk[a] = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
  const uint32_t p2bot = V == FS_P2_BOT ? 1u : 0u;
  const uint32_t h = A.rec_count | (A.rec0 << 15) | (A.rec1 << 18) | (A.act0 << 21) | (A.act1 << 24) |
                     (A.pending << 27) | (A.has_term << 28) | (p2bot << 29);
  s.aw[a] = make_int2(A.frame_count, (int)h);
  s.cum[a] = A.cum;
  if constexpr (V == FS_P2_BOT) {
    const Bot1& b = A.bot;
    s.rng[a] = b.rng;
    s.bot[a] = make_uint2(b.mplan | (b.midx << 3) | (b.aplan << 10) | (b.aidx << 13) | (b.prev_opp << 20) |
                              (1u << 25) | (A.bin << 26),
                          __float_as_uint(b.prev_dist));
  }
}

// UpdatePushCharacterVsCharacter (BC:483-501), Rect semantics, both fighters on one lane.  The
// pair kernel's test, (xmax_o > px) & (o_px < xmax_m), is the same expression on both lanes, and
// the two shifts are -d/2 and +d/2 of the one distance d (the left fighter moves left), computed
// before either fighter moves: the values push_character_vs_character gives each lane.
template <int FM>
__device__ __forceinline__ void push_character_vs_character1(Fighter& f0, Fighter& f1) {
  const float xmax0 = fadd<FM>(f0.pw, f0.px), xmax1 = fadd<FM>(f1.pw, f1.px);  // Rect.xMax = width + x
  const bool overlap = (xmax1 > f0.px) & (f1.px < xmax0);
  if (!overlap || f0.x == f1.x) return;  // a tie pushes nothing (BC:490-499)
  const bool left0 = f0.x < f1.x;        // fighter 0 is the left one
  float dx0, dx1;
  if constexpr (FM == FS_FLOAT_DOUBLE) {
    const double d = left0 ? (double)xmax0 - (double)f1.px : (double)xmax1 - (double)f0.px;
    const float neg = (float)(d * -1 / 2), pos = (float)(d * 1 / 2);
    dx0 = left0 ? neg : pos;
    dx1 = left0 ? pos : neg;
  } else {
    const float d = left0 ? __fsub_rn(xmax0, f1.px) : __fsub_rn(xmax1, f0.px);
    const float neg = d * -1.0f / 2.0f, pos = d * 1.0f / 2.0f;
    dx0 = left0 ? neg : pos;
    dx1 = left0 ? pos : neg;
  }
  apply_position_change<FM>(f0, dx0);
  apply_position_change<FM>(f1, dx1);
}

// The resolution entry's nibble for overlap mask m: the outcome at the attacker's hit count (low
// nibble) and at 0 (high), as hitbox_hurtbox_collision picks it
__device__ __forceinline__ uint32_t resolve_byte(U4 res, uint32_t m) {
  const uint32_t sel = (m & 7u) | 0x0c0c0c00u;
  const uint32_t lo = __builtin_amdgcn_perm(res.y, res.x, sel), hi = __builtin_amdgcn_perm(res.w, res.z, sel);
  return (m & 8u) ? hi : lo;
}

// UpdateHitboxHurtboxCollision (BC:521-591) for both phases on one lane: phase A (P1 attacks, P2
// defends) at P1's hit count, phase B (P2 attacks P1) at P2's hit count after phase A (0 if A hit,
// SetCurrentAction), then the defenders' NotifyDamaged, the attackers' NotifyAttackHit, the
// proximity latches and SetHitStun on both fighters, in hitbox_hurtbox_collision's order.
template <int FM>
__device__ __forceinline__ void hitbox_hurtbox_collision1(Fighter& f0, Fighter& f1, const RecGeo& R0,
                                                          const RecGeo& R1, U4 resA, U4 resB, uint32_t ymA,
                                                          uint32_t ymB) {
  const uint32_t xmA = box_x_overlaps<FM>(R0.hit.z, R0.hit.w, f0.hx0, f0.hx1, R1.hurt.zw, F2{f1.ux0, f1.ux1});
  const uint32_t xmB = box_x_overlaps<FM>(R1.hit.z, R1.hit.w, f1.hx0, f1.hx1, R0.hurt.zw, F2{f0.ux0, f0.ux1});
  const uint32_t tA = resolve_byte(resA, xmA & ymA) & 15u;
  const uint32_t hitA = tA & 1u;
  const uint32_t tabB = resolve_byte(resB, xmB & ymB);
  const uint32_t tB = hitA ? (tabB >> 4) : (tabB & 15u);
  const bool hit0 = (tB & 1u) != 0, hit1 = hitA != 0;  // P1 is phase B's defender, P2 phase A's
  f0.hits += (int)hitA;                                // NotifyAttackHit for P1 (F:352-355)
  int stun0 = 0, stun1 = 0;
  if (hit0) {
    const AttackInfo ad = attack_info((int)((tB >> 1) & 3u));
    const int res = notify_damaged(f0, ad);
    stun0 = res == DR_GUARD ? ad.guard_stun : res == DR_GUARD_BREAK ? ad.guard_break_stun : ad.hit_stun;
  }
  if (!hit0 && ((tB >> 3) & 1u) && f0.in_back) f0.prox = true;  // NotifyInProximityGuardRange (F:400-406)
  if (hit1) {
    const AttackInfo ad = attack_info((int)((tA >> 1) & 3u));
    const int res = notify_damaged(f1, ad);
    stun1 = res == DR_GUARD ? ad.guard_stun : res == DR_GUARD_BREAK ? ad.guard_break_stun : ad.hit_stun;
  }
  if (!hit1 && ((tA >> 3) & 1u) && f1.in_back) f1.prox = true;
  f1.hits += hit0 ? 1 : 0;  // NotifyAttackHit for P2
  // SetHitStun on both, phase B last (BC:576-578)
  const int sA0 = hit1 ? stun1 : f0.stun, sA1 = hit1 ? stun1 : f1.stun;
  f0.stun = hit0 ? stun0 : sA0;
  f1.stun = hit0 ? stun0 : sA1;
}

// the reset burst (reset_burst) for both fighters of the arena
template <int FM, int V>
__device__ __forceinline__ void reset_burst1(Arena1& A, bool after_ko) {
  constexpr bool BOT = V == FS_P2_BOT;
  if (after_ko) {
    const int v0 = A.f0.vital, v1 = A.f1.vital;
    end_tick(A.f0, A.f0.won || (v0 > 0 && v1 <= 0));  // a sole survivor wins (BC:310-323)
    end_tick(A.f1, A.f1.won || (v1 > 0 && v0 <= 0));
  }
  setup_battle_start(A.f0, kP1StartX);
  setup_battle_start(A.f1, kP2StartX);
  const float x1 = A.f0.x, x2 = A.f1.x;
  const uint32_t p1_act = (uint32_t)A.f0.act;
  if constexpr (BOT) {  // BattleAI.Reset (AI:393-403)
    A.bot.mplan = A.bot.midx = A.bot.aplan = A.bot.aidx = 0;
    A.bot.prev_dist = bot_distance<FM>(x1, x2);
    A.bot.prev_opp = p1_act;
  }
  const uint32_t in0 = A.act0;
  const uint32_t in1 = BOT ? A.bin : (V == FS_P2_NOOP ? 0u : A.act1);
  if (A.rec_count < kMaxRecording) {  // RecordInput in the Intro tick (BC:333)
    A.rec0 = in0;
    A.rec1 = in1;
    A.rec_count++;
  }
  auto intro = [](Fighter& f, uint32_t in, int k) {
    const uint32_t r = rel_bits(in, k);
    f.hist = (r & 1) | ((r & 2) << 15);
    f.hold = (in & IN_ATTACK) ? 1 : 0;
    const bool stunned = f.stun > 0;
    f.stun -= stunned ? 1 : 0;
    f.frame = stunned ? 0 : 1;
  };
  intro(A.f0, in0, 0);
  intro(A.f1, in1, 1);
  A.frame_count = -1;
  A.rec_count = 0;
  if constexpr (BOT) A.bin = bot_next_input1(A.bot, bot_distance<FM>(x1, x2), p1_act, bot_prefetch1(A.bot));
}

// outputs (FE:336-380, 537-549): a lane stores both fighters' values of each [N][2] array at once
__device__ __forceinline__ uint32_t obs_move(const Fighter& f) {
  const int a = f.act;
  return (a == A_DEAD || a == A_WIN) ? (uint32_t)A_STAND : (uint32_t)a;  // FE:537-549
}
__device__ __forceinline__ float obs_move_frame(const Fighter& f) {
  const int a = (f.act == A_DEAD || f.act == A_WIN) ? A_STAND : f.act;
  return (float)((a == A_STAND || a == A_FORWARD || a == A_BACKWARD) ? 0 : f.frame);  // FE:339-358
}
__device__ __forceinline__ void write_obs1(const Arena1& A, uint8_t* guard, uint8_t* move, float* move_frame,
                                           float* position, int32_t* frame, uint8_t* action, uint8_t* hitstun,
                                           uint32_t r) {
  const bool recd = A.rec_count > 0;
  st_off(reinterpret_cast<uint16_t*>(guard), 2 * r, (uint16_t)(A.f0.guard | (A.f1.guard << 8)));
  st_off(reinterpret_cast<uint16_t*>(move), 2 * r, (uint16_t)(obs_move(A.f0) | (obs_move(A.f1) << 8)));
  st_off(reinterpret_cast<F2*>(move_frame), 8 * r, F2{obs_move_frame(A.f0), obs_move_frame(A.f1)});
  st_off(reinterpret_cast<F2*>(position), 8 * r, F2{A.f0.x, A.f1.x});
  st_off(reinterpret_cast<uint16_t*>(action), 2 * r, (uint16_t)(recd ? (A.rec0 | (A.rec1 << 8)) : 0u));
  st_off(reinterpret_cast<uint16_t*>(hitstun), 2 * r, (uint16_t)((A.f0.stun & 0xff) | ((A.f1.stun & 0xff) << 8)));
  st_off(frame, 4 * r, (int32_t)A.frame_count);
}
__device__ __forceinline__ void write_main1(const Arena1& A, const DevOutputs& o, uint32_t r) {
  write_obs1(A, o.guard, o.move, o.move_frame, o.position, o.frame, o.action, o.hitstun, r);
}
__device__ __forceinline__ void write_final1(const Arena1& A, const DevOutputs& o, uint32_t r) {
  write_obs1(A, o.final_guard, o.final_move, o.final_move_frame, o.final_position, o.final_frame, o.final_action,
             o.final_hitstun, r);
}

// fs_step_n_packed: the two lane records of the arena (include/footsies.h fs_packed_traj, the
// layout packed_record writes from the two-lane kernel) at records 2 r and 2 r + 1, as two 16-B
// stores; w3 of P1's record is the frame, of P2's the terminated byte (0 in a final record).
__device__ __forceinline__ PkRec packed_record1(const Fighter& f, uint32_t rec_count, uint32_t rec, uint32_t w3) {
  PkRec v;
  const uint32_t act = rec_count > 0 ? rec : 0u;  // a 3-bit input
  v.x = (uint32_t)f.guard | (obs_move(f) << 8) | (act << 16) | ((uint32_t)f.stun << 24);
  v.y = __float_as_uint(obs_move_frame(f));
  v.z = __float_as_uint(f.x);
  v.w = w3;
  return v;
}
__device__ __forceinline__ void write_packed1(const Arena1& A, uint4* base, uint32_t r, uint32_t w3_p2) {
  st_off(reinterpret_cast<PkRec*>(base), 32u * r, packed_record1(A.f0, A.rec_count, A.rec0, (uint32_t)A.frame_count));
  st_off(reinterpret_cast<PkRec*>(base), 32u * r + 16u, packed_record1(A.f1, A.rec_count, A.rec1, w3_p2));
}

// (see opaque_burst_results)
__device__ __forceinline__ void opaque_burst_results1(Arena1& A) {
  asm volatile("" : "+v"(A.f0.x), "+v"(A.f0.act), "+v"(A.f0.frame), "+v"(A.f0.vital), "+v"(A.f0.guard),
               "+v"(A.f0.hits), "+v"(A.f0.buf), "+v"(A.f0.rsv), "+v"(A.f0.hold), "+v"(A.f0.won), "+v"(A.f0.hist));
  asm volatile("" : "+v"(A.f1.x), "+v"(A.f1.act), "+v"(A.f1.frame), "+v"(A.f1.vital), "+v"(A.f1.guard),
               "+v"(A.f1.hits), "+v"(A.f1.buf), "+v"(A.f1.rsv), "+v"(A.f1.hold), "+v"(A.f1.won), "+v"(A.f1.hist));
  asm volatile("" : "+v"(A.ai0), "+v"(A.ai1), "+v"(A.cum), "+v"(A.pending), "+v"(A.has_term), "+v"(A.frame_count),
               "+v"(A.rec_count));
}

// The row pair of the next tick (P1's, P2's), made resident before this tick's stores: the
// s_waitcnt and both copies in one statement (see row_load / settle_w).
template <int WAIT>
__device__ __forceinline__ void settle2(uint32_t& n1, uint32_t& n2) {
  uint32_t r1, r2;
  asm volatile("s_waitcnt vmcnt(%4)\n\tv_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=v"(r1), "=v"(r2)
               : "v"(n1), "v"(n2), "n"(WAIT) : "memory");
  n1 = r1;
  n2 = r2;
}

// one env-step of one arena: env_step's phases for both fighters
template <int FM, int P2, int WAIT, bool PK>
__device__ __forceinline__ void env_step1(Arena1& A, uint32_t a1, uint32_t a2, const StepParams& p, uint32_t r,
                                          uint32_t& n1, uint32_t& n2) {
  constexpr bool BOT = P2 == FS_P2_BOT;
  const DevOutputs& o = p.out;
  if (A.pending) {  // FS_AUTORESET_NEXT_STEP: this step runs the reset burst only
    reset_burst1<FM, P2>(A, true);
    A.pending = 0;
    A.has_term = 0;
    A.cum = 0.0;
    A.ai0 = A.ai1 = stand_info();
    settle2<WAIT>(n1, n2);
    if constexpr (PK) {
      write_packed1(A, o.pk_lanes, r, 0u);
      st_off(o.reward, 8 * r, 0.0);
    } else {
      write_main1(A, o, r);
      st_off(o.reward, 8 * r, 0.0);
      st_off(o.terminated, r, (uint8_t)0);
      st_off(o.truncated, r, (uint8_t)0);
    }
    opaque_burst_results1(A);
    return;
  }
  // the actor inputs of this frame (BC:383-447)
  A.act0 = a1;
  if constexpr (P2 == FS_P2_EXTERNAL) A.act1 = a2;
  const uint32_t in0 = A.act0;
  const uint32_t in1 = BOT ? A.bin : (P2 == FS_P2_NOOP ? 0u : A.act1);
  const int gb0 = A.f0.guard, gb1 = A.f1.guard;  // guards of FE._current_state
  BotPre1 bpre;
  if constexpr (BOT) bpre = bot_prefetch1(A.bot);
  A.frame_count++;
  if (A.rec_count < kMaxRecording) {  // RecordInput (BC:593-607)
    A.rec0 = in0;
    A.rec1 = in1;
    A.rec_count++;
  }
  const InputEval e0 = update_input(A.f0, in0, kRelLut0);
  const InputEval e1 = update_input(A.f1, in1, kRelLut1);
  const AInfo ai0 = A.ai0, ai1 = A.ai1;
  increment_action_frame(A.f0, ai0);
  increment_action_frame(A.f1, ai1);
  // both fighters' request entries and continuing records in flight together: the selects are
  // made opaque so that neither chain is sunk into a branch (which would serialize the reads)
  bool keep0, keep1;
  uint32_t sel0 = request_sel(A.f0, e0, ai0, keep0), sel1 = request_sel(A.f1, e1, ai1, keep1);
  asm volatile("" : "+v"(sel0), "+v"(sel1));
  const uint32_t q0 = sT.req_table[sel0], q1 = sT.req_table[sel1];
  const int rc0 = frame_record<false>(A.f0), rc1 = frame_record<false>(A.f1);
  uint32_t rs0, rs1;
  const bool set0 = apply_request(A.f0, q0, keep0, e0, &rs0);
  const bool set1 = apply_request(A.f1, q1, keep1, e1, &rs1);
  A.f0.rec = set0 ? (int)rs0 : rc0;
  A.f1.rec = set1 ? (int)rs1 : rc1;
  // every table read of the rest of the tick in one round trip (the y-overlap bits and the
  // resolution entries first: their addresses are ready as soon as the records are)
  const uint32_t ymA = sT.ybits[((uint32_t)A.f0.rec << 6) | (uint32_t)A.f1.rec];  // P1's hitboxes on P2
  const uint32_t ymB = sT.ybits[((uint32_t)A.f1.rec << 6) | (uint32_t)A.f0.rec];
  const U4 resA = reinterpret_cast<const U4*>(sT.resolve)[__umul24((uint32_t)A.f0.hits, (uint32_t)kNumFrameRecs) +
                                                          (uint32_t)A.f0.rec];
  const U4 resB = reinterpret_cast<const U4*>(sT.resolve)[__umul24((uint32_t)A.f1.hits, (uint32_t)kNumFrameRecs) +
                                                          (uint32_t)A.f1.rec];
  const RecGeo R0 = frame_rec<false>(0, (uint32_t)A.f0.rec);
  const RecGeo R1 = frame_rec<false>(1, (uint32_t)A.f1.rec);
  update_movement<FM>(A.f0, R0.push.z);
  update_movement<FM>(A.f1, R1.push.z);
  update_boxes<FM>(A.f0, R0);
  update_boxes<FM>(A.f1, R1);
  push_character_vs_character1<FM>(A.f0, A.f1);
  push_character_vs_background<FM>(A.f0);
  push_character_vs_background<FM>(A.f1);
  asm volatile("" ::"v"(R0.push), "v"(R0.hurt), "v"(R0.hit), "v"(R1.push), "v"(R1.hurt), "v"(R1.hit), "v"(resA),
               "v"(resB), "v"(ymA), "v"(ymB));
  hitbox_hurtbox_collision1<FM>(A.f0, A.f1, R0, R1, resA, resB, ymA, ymB);
  A.ai0 = action_info<false>(A.f0.act);  // the next tick's ActionInfo, read early
  A.ai1 = action_info<false>(A.f1.act);
  // KO check (BC:212-213) and reward (FE:382-405): per fighter, bit 0 = vital 0, bit 1 = guard dropped
  const uint32_t fl1 = ((uint32_t)(A.f0.vital - 1) >> 31) | (((uint32_t)(A.f0.guard - gb0) >> 31) << 1);
  const uint32_t fl2 = ((uint32_t)(A.f1.vital - 1) >> 31) | (((uint32_t)(A.f1.guard - gb1) >> 31) << 1);
  const uint32_t any_fl = fl1 | fl2;
  const bool over = (any_fl & 1u) != 0;
  double reward = 0.0;
  if (p.dense_reward) {
    if (any_fl != 0) {
      if (fl1 & 2u) reward -= 0.3;
      if (fl2 & 2u) reward += 0.3;
      A.cum += reward;
      if (over) reward += (double)((fl2 & 1u) ? 1 : -1) - A.cum;
    }
  } else {
    reward = over ? ((fl2 & 1u) ? 1.0 : -1.0) : 0.0;
  }
  settle2<WAIT>(n1, n2);
  if (over) {
    A.f0.hist = A.f1.hist = 0;  // ChangeRoundState(KO): ClearInput (BC:296-299)
    A.f0.hold = A.f1.hold = 0;
    if (p.autoreset_mode == FS_AUTORESET_SAME_STEP) {
      if constexpr (PK) write_packed1(A, o.pk_final, r, 0u);
      else write_final1(A, o, r);
      reset_burst1<FM, P2>(A, true);
      A.cum = 0.0;
      A.has_term = 0;
      A.ai0 = A.ai1 = stand_info();
    } else {
      A.pending = 1;
      A.has_term = 1;
    }
  } else {
    if constexpr (BOT)  // TrainingManager.Step -> RequestNextInput -> getNextAIInput
      A.bin = bot_next_input1(A.bot, bot_distance<FM>(A.f0.x, A.f1.x), (uint32_t)A.f0.act, bpre);
    A.has_term = 0;
  }
  if constexpr (PK) {
    write_packed1(A, o.pk_lanes, r, over ? 1u : 0u);
    st_off(o.reward, 8 * r, reward);
  } else {
    write_main1(A, o, r);
    st_off(o.reward, 8 * r, reward);
    st_off(o.terminated, r, (uint8_t)(over ? 1 : 0));
    st_off(o.truncated, r, (uint8_t)0);
  }
  asm volatile("" ::"v"(A.ai0), "v"(A.ai1));
}

// The fused rollout, one lane per arena.  Both action rows of tick t + D are issued at the top of
// tick t (two untracked loads into the slot of tick t's rows, D slots in all), and before tick t's
// stores the wave waits for tick t + 1's rows with vmcnt(12 (D - 1)): ticks t + 1 - D .. t - 1 issued
// 10 output stores and 2 row loads each after them (tools/check_async_loads.py proves the count on
// the assembly).  Packed trajectories (PK): 3 stores per tick (the two lane records and the
// reward), so vmcnt(5 (D - 1)).  Loads and stores retire in order on gfx9, so that wait also needs the stores of
// tick t - D to be acknowledged: a deeper pipeline asks for older stores only.
#ifndef FS_ROW_DEPTH
#define FS_ROW_DEPTH 3
#endif
#ifndef FS_ROW_DEPTH_PK
#define FS_ROW_DEPTH_PK FS_ROW_DEPTH
#endif
template <int FM, int P2, bool PK>
__device__ __forceinline__ void step_body1(const StepParams& p) {
  constexpr int D = PK ? FS_ROW_DEPTH_PK : FS_ROW_DEPTH;
  constexpr int W = (PK ? 5 : 12) * (D - 1);
  // (the main loop below unrolls at most four ticks per iteration and the remainder handles at most
  // three, so a deeper pipeline would skip ticks; vmcnt's 6-bit field bounds W as well)
  static_assert(D >= 2 && D <= 4 && W <= 63, "row pipeline depth 2..4");
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = a < p.n_envs;
  const int ar = active ? a : 0;
  Arena1 A;
  load_arena1<P2>(A, p.st, ar);
  // P2's rows exist only for a remote P2; otherwise the second load re-reads P1's row (ignored)
  const uint8_t* src2 = P2 == FS_P2_EXTERNAL ? p.p2 : p.p1;
  const int n = p.n_steps, last = n - 1;
  const uint32_t N = (uint32_t)p.n_envs;
  auto issue1 = [&](int t) -> uint32_t { return row_load(p.p1 + (uint32_t)min(t, last) * N + (uint32_t)ar); };
  auto issue2 = [&](int t) -> uint32_t { return row_load(src2 + (uint32_t)min(t, last) * N + (uint32_t)ar); };
  uint32_t fl1[D], fl2[D];  // the slots: rows in flight (read only by their wait)
#pragma unroll
  for (int j = 0; j < D; j++) {
    fl1[j] = issue1(j);
    fl2[j] = issue2(j);
  }
  stage_tables<P2 == FS_P2_BOT>();
  if (!active) {
#pragma unroll
    for (int j = 0; j < D; j++) asm volatile("s_waitcnt vmcnt(0)" ::"v"(fl1[j]), "v"(fl2[j]) : "memory");
    return;
  }
  A.ai0 = action_info<false>(A.f0.act);
  A.ai1 = action_info<false>(A.f1.act);
  const uint32_t row_step = (uint32_t)p.out_stride_steps * N;
  uint32_t rd1, rd2;  // the rows of the current tick, resident
  asm volatile("s_waitcnt vmcnt(0)\n\tv_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=v"(rd1), "=v"(rd2)
               : "v"(fl1[0]), "v"(fl2[0]) : "memory");
  // (the other slots are resident too; one copy each tells tools/check_async_loads.py so, which
  // needs it when the launch is shorter than the pipeline)
#pragma unroll
  for (int j = 1; j < D; j++) {
    uint32_t c1, c2;
    asm volatile("s_waitcnt vmcnt(0)\n\tv_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=v"(c1), "=v"(c2)
                 : "v"(fl1[j]), "v"(fl2[j]) : "memory");
  }
  // one tick in slot J = t mod D (a compile-time index, so the slots stay in registers)
  // time-sliced wave priority (prio_slice), as in the two-lane loop: at two waves per SIMD (131 072
  // arenas) it keeps a SIMD's waves progressing together (fs_kernels.hip one_lane_prio)
  const uint32_t grp = prio_group();
  auto tick = [&](int t, auto J) {
    constexpr int j = decltype(J)::value, jn = (j + 1) % D;
    fl1[j] = issue1(t + D);
    fl2[j] = issue2(t + D);
    if (p.prio) prio_slice(grp);
    uint32_t n1 = fl1[jn], n2 = fl2[jn];
    env_step1<FM, P2, W, PK>(A, rd1 & 7u, rd2 & 7u, p, (uint32_t)t * row_step + (uint32_t)a, n1, n2);
    rd1 = n1;
    rd2 = n2;
  };
  int t = 0;
  for (; t + D <= n; t += D) {
    tick(t, std::integral_constant<int, 0>{});
    tick(t + 1, std::integral_constant<int, 1>{});
    if constexpr (D > 2) tick(t + 2, std::integral_constant<int, 2 % D>{});
    if constexpr (D > 3) tick(t + 3, std::integral_constant<int, 3 % D>{});
  }
  // the remaining n mod D ticks, slots 0 .. D - 2 (their waits re-read rows clamped to the last)
  // (nested, so that no path of the code runs a later remainder tick without the earlier ones)
  if (t < n) {
    tick(t, std::integral_constant<int, 0>{});
    if (t + 1 < n) {
      tick(t + 1, std::integral_constant<int, 1 % D>{});
      if constexpr (D > 3) {
        if (t + 2 < n) tick(t + 2, std::integral_constant<int, 2 % D>{});
      }
    }
  }
#pragma unroll
  for (int j = 0; j < D; j++) asm volatile("s_waitcnt vmcnt(0)" ::"v"(fl1[j]), "v"(fl2[j]) : "memory");
  store_arena1<P2>(A, p.st, a);
}

template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n1(StepParams p) {
  step_body1<FM, P2, false>(p);
}

// fs_step_n_packed with one lane per arena (the launches k_step_n1 takes, packed records)
template <int FM, int P2>
__global__ __launch_bounds__(256) void k_step_n1_packed(StepParams p) {
  step_body1<FM, P2, true>(p);
}
