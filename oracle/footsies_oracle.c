/*
 * footsies_oracle.c -- CPU ORACLE.  TEST INFRASTRUCTURE ONLY.
 *
 * A scalar, from-scratch C restatement of the reference FOOTSIES simulation, used
 * (a) as the checker the HIP path is compared against in tests/ and smoke(), and
 * (b) as bench.py's `cpu_baseline` leg.  The product path (libfootsies.so) never
 * links, loads or calls this file.
 *
 * It deliberately keeps the reference's *structure* rather than the kernel's:
 * the round-state machine with its timers (BattleCore.cs:138-327), the 180-deep
 * input/inputDown/inputUp histories (Fighter.cs:98-101, 172-188), window scans
 * over the ActionData lists (ActionData.cs:87-168), boxes materialised as lists
 * and shifted by ApplyPositionChange (Fighter.cs:331-350), the bot's real
 * queues and 10-entry FightState array (BattleAI.cs:26-32, 344-363), and the
 * FootsiesEnv post-processing driven from a stored previous EnvironmentState
 * (footsies.py:518-570).  The kernel's bit-packed state, dense tables and
 * (plan,index) bot encoding are therefore checked against an independent form.
 *
 * Parity status: the C# path cannot be compiled or run here (no Unity / Mono /
 * .NET, no game binary) and the reference ships no fixtures, so the simulation
 * semantics are pinned only by hand-derived known-answer tests; the Python
 * post-processing is pinned by golden vectors produced by the reference's own
 * FootsiesEnv methods (tests/golden/).  Unity engine internals it depends on --
 * Rect.Overlaps/xMax, Random (Xorshift128), and the Mono float evaluation
 * precision -- are restated from their published behaviour and are
 * "parity unpinned" (see DESIGN.md).
 *
 * Paths below are relative to the reference root; BC = Assets/Script/BattleCore.cs,
 * F = Assets/Script/Fighter.cs, AD = Assets/Script/ActionData.cs,
 * AI = Assets/Script/BattleAI.cs, FE = footsies-gym/footsies_gym/envs/footsies.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/footsies.h"
#include "or_tables.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_EXPORT __attribute__((visibility("default")))

/* CommonActionID (F:42-61) */
enum { STAND = 0, FORWARD = 1, BACKWARD = 2, DASH_FORWARD = 10, DASH_BACKWARD = 11, N_ATTACK = 100,
       B_ATTACK = 105, N_SPECIAL = 110, B_SPECIAL = 115, DAMAGE = 200, GUARD_M = 301, GUARD_STAND = 305,
       GUARD_CROUCH = 306, GUARD_BREAK = 310, GUARD_PROXIMITY = 350, DEAD = 500, WIN = 510 };
/* InputDefine (InputData.cs:8-14) */
enum { IN_LEFT = 1, IN_RIGHT = 2, IN_ATTACK = 4 };
/* ActionType (AD:60-66) */
enum { TYPE_MOVEMENT = 0, TYPE_ATTACK = 1, TYPE_DAMAGE = 2, TYPE_GUARD = 3 };
/* DamageResult (F:63-69) */
enum { DR_DAMAGE = 1, DR_GUARD = 2, DR_GUARD_BREAK = 3 };
/* RoundStateType (BC:13-20) */
enum { RS_STOP, RS_INTRO, RS_FIGHT, RS_KO, RS_END };

/* ------------------------------------------------------------------------ */
/* float evaluation model                                                    */
/* ------------------------------------------------------------------------ */
/* FS_FLOAT_STRICT32: each C# float operation rounds to binary32 (compile with
 * -ffp-contract=off, SSE2).  FS_FLOAT_DOUBLE: a whole C# expression is evaluated
 * in binary64 and rounded once where it is stored into a float field, passed as
 * a float argument or returned from a float property. */
/* pos + rx*sign  (TransformToFightRect, F:706-719) */
static inline float x_plus_rel(int mode, float base, float rx, int sign) {
  if (mode == FS_FLOAT_DOUBLE) return (float)((double)base + (double)rx * (double)sign);
  float t = rx * (float)sign;
  return base + t;
}
/* a + b as one rounded float store */
static inline float fadd(int mode, float a, float b) {
  if (mode == FS_FLOAT_DOUBLE) return (float)((double)a + (double)b);
  return a + b;
}
static inline float fsub(int mode, float a, float b) {
  if (mode == FS_FLOAT_DOUBLE) return (float)((double)a - (double)b);
  return a - b;
}
/* position.x += speed * sign * Time.deltaTime  (F:300, 316) */
static inline float pos_plus_vel(int mode, float pos, float v, int sign) {
  if (mode == FS_FLOAT_DOUBLE) return (float)((double)pos + (double)v * (double)sign * (double)OR_FIXED_DT);
  float t = v * (float)sign;
  t = t * OR_FIXED_DT;
  return pos + t;
}
/* position.x -= speed * sign * Time.deltaTime  (F:305) */
static inline float pos_minus_vel(int mode, float pos, float v, int sign) {
  if (mode == FS_FLOAT_DOUBLE) return (float)((double)pos - (double)v * (double)sign * (double)OR_FIXED_DT);
  float t = v * (float)sign;
  t = t * OR_FIXED_DT;
  return pos - t;
}

/* ------------------------------------------------------------------------ */
/* UnityEngine.Random (engine code; Xorshift128 per public reverse-engineering) */
/* ------------------------------------------------------------------------ */
static void rng_init(uint32_t s[4], int32_t seed) {
  s[0] = (uint32_t)seed;
  s[1] = s[0] * 1812433253u + 1u;
  s[2] = s[1] * 1812433253u + 1u;
  s[3] = s[2] * 1812433253u + 1u;
}
static uint32_t rng_next(uint32_t s[4]) {
  uint32_t t = s[0] ^ (s[0] << 11);
  s[0] = s[1];
  s[1] = s[2];
  s[2] = s[3];
  s[3] = s[3] ^ (s[3] >> 19) ^ t ^ (t >> 8);
  return s[3];
}
/* Random.Range(int min, int max), max exclusive */
static int rng_range(uint32_t s[4], int mn, int mx) {
  uint32_t r = rng_next(s);
  return mn + (int)(r % (uint32_t)(mx - mn));
}

/* ------------------------------------------------------------------------ */
/* types                                                                     */
/* ------------------------------------------------------------------------ */
/* UnityEngine.Rect: (x, y, width, height).  Rect methods treat x as xMin;
 * BoxBase (F:8-26) treats x as the centre. */
typedef struct { float x, y, w, h; } rect_t;
typedef struct { rect_t rect; int proximity; int attack_id; } hitbox_t;

typedef struct {
  float pos_x, pos_y;
  float velocity_x;
  int is_face_right;
  hitbox_t hitboxes[4];
  int n_hitboxes;
  rect_t hurtboxes[4];
  int n_hurtboxes;
  rect_t pushbox;
  int vital, guard;
  int action_id, action_frame, hit_count, hitstun;
  /* 180-frame histories (F:98-101), kept as a ring: element i lives at (head + i) % 180 */
  int in[OR_INPUT_RECORD_FRAME], in_down[OR_INPUT_RECORD_FRAME], in_up[OR_INPUT_RECORD_FRAME];
  int head;
  int is_input_backward, is_reserve_proximity_guard;
  int buffer_action_id, reserve_damage_action_id;
  int sprite_shake;
  int has_won;
} fighter_t;

typedef struct {
  int valid;
  float distance_x;
  int opp_damage, opp_guard_break, opp_blocking, opp_normal_attack, opp_special_attack;
  int opp_action; /* kept for the canonical export */
} fight_state_t;

typedef struct { int q[128]; int head, count; } queue_t;

typedef struct {
  queue_t move_q, attack_q;
  fight_state_t fs[10]; /* maxFightStateRecord (AI:30-32) */
  int move_plan, move_len, attack_plan, attack_len; /* canonical export only */
} bot_t;

typedef struct {
  fighter_t f[2];
  int round_state;
  float timer;
  int frame_count;
  uint32_t rec_idx;          /* currentRecordingInputIndex (BC:70) */
  int rec_last[2];           /* recordingPnInput[rec_idx - 1].input */
  int actor_in[2];           /* TrainingRemoteActor.input of the remote P1 / P2 actors */
  int bot_in[2];             /* TrainingBattleAIActor.input of P1's / P2's bot */
  int p2_bot;                /* TrainingManager.actorP2 is the bot (BC:158-167) */
  uint32_t rng[4];           /* the game's one UnityEngine.Random, shared by both bots */
  bot_t bot[2];              /* P1's BattleAI (isPlayer1, by_example) and P2's */
  /* FootsiesEnv side */
  fs_env_state cur_state;    /* FE._current_state */
  double cum_reward;         /* FE._cummulative_episode_reward */
  int has_terminated;        /* FE.has_terminated */
  int reset_pending;         /* FS_AUTORESET_NEXT_STEP */
  fs_env_state* dq;          /* FE.delayed_frame_queue (FE:129-131), capacity frame_delay + 1 */
  int dq_head, dq_count;
  /* emission bookkeeping of one driver call */
  int emitted;
  int emitted_battle_over;
  fs_env_state emitted_state;
} arena_t;

typedef struct or_ctx {
  fs_config cfg;
  int n;
  arena_t* a;
  /* host outputs */
  uint8_t *guard, *move, *action, *hitstun, *terminated, *truncated;
  float *move_frame, *position;
  double* reward;
  int32_t* frame;
  uint8_t *f_guard, *f_move, *f_action, *f_hitstun;
  float *f_move_frame, *f_position;
  int32_t* f_frame;
  uint64_t steps;
} or_ctx;
typedef or_ctx* or_handle;

/* ------------------------------------------------------------------------ */
/* frame data lookups (AD:87-168; FighterData dictionaries FighterData.cs:48-78) */
/* ------------------------------------------------------------------------ */
static const or_action_data* action_data(int id) {
  for (int i = 0; i < OR_N_ACTIONS; i++)
    if (OR_ACTIONS[i].id == id) return &OR_ACTIONS[i];
  abort();
}
static const or_attack_data* attack_data(int id) {
  for (int i = 0; i < OR_N_ATTACKS; i++)
    if (OR_ATTACKS[i].id == id) return &OR_ATTACKS[i];
  return 0;
}
static int move_index(int id) { /* FOOTSIES_MOVE_ID_TO_INDEX (moves.py:41-42): enum order == id order */
  for (int i = 0; i < OR_N_ACTIONS; i++)
    if (OR_ACTIONS[i].id == id) return i;
  abort();
}
static inline int in_window(int s, int e, int frame) { return frame >= s && frame <= e; }

/* ------------------------------------------------------------------------ */
/* Fighter (F:71-812)                                                        */
/* ------------------------------------------------------------------------ */
static inline int hist_in(const fighter_t* f, int i) { return f->in[(f->head + i) % OR_INPUT_RECORD_FRAME]; }

static int is_action_end(const fighter_t* f) { return f->action_frame >= action_data(f->action_id)->frame_count; }

static void clear_input(fighter_t* f) { /* F:521-529 */
  memset(f->in, 0, sizeof f->in);
  memset(f->in_down, 0, sizeof f->in_down);
  memset(f->in_up, 0, sizeof f->in_up);
}

static void set_current_action(fighter_t* f, int id, int start_frame) { /* F:546-563 */
  f->action_id = id;
  f->action_frame = start_frame;
  f->hit_count = 0;
  f->buffer_action_id = -1;
  f->reserve_damage_action_id = -1;
  f->sprite_shake = 0;
}

static void setup_battle_start(fighter_t* f, float start_x, int is_player_one) { /* F:120-135 */
  f->pos_x = start_x;
  f->pos_y = 0.0f;
  f->is_face_right = is_player_one;
  f->vital = 1;
  f->guard = OR_START_GUARD_HEALTH;
  f->has_won = 0;
  f->velocity_x = 0.0f;
  clear_input(f);
  set_current_action(f, STAND, 0);
}

static void increment_action_frame(fighter_t* f) { /* F:140-166 */
  if (abs(f->sprite_shake) > 0) {
    f->sprite_shake *= -1;
    f->sprite_shake += (f->sprite_shake > 0 ? -1 : 1);
  }
  if (f->hitstun > 0) {
    f->hitstun--;
    return;
  }
  f->action_frame++;
  if (is_action_end(f)) {
    const or_action_data* ad = action_data(f->action_id);
    if (ad->is_loop) f->action_frame = ad->loop_from;
  }
}

static void update_input(fighter_t* f, int input) { /* F:172-188 */
  f->head = (f->head + OR_INPUT_RECORD_FRAME - 1) % OR_INPUT_RECORD_FRAME; /* shift by one frame */
  int h0 = f->head, h1 = (f->head + 1) % OR_INPUT_RECORD_FRAME;
  f->in[h0] = input;
  f->in_down[h0] = (f->in[h0] ^ f->in[h1]) & f->in[h0];
  f->in_up[h0] = (f->in[h0] ^ f->in[h1]) & ~f->in[h0];
}

static int is_attack_input(int in) { return (in & IN_ATTACK) > 0; } /* F:637-640 */
static int is_forward_input(const fighter_t* f, int in) { /* F:642-653 */
  return f->is_face_right ? (in & IN_RIGHT) > 0 : (in & IN_LEFT) > 0;
}
static int is_backward_input(const fighter_t* f, int in) { /* F:655-666 */
  return f->is_face_right ? (in & IN_LEFT) > 0 : (in & IN_RIGHT) > 0;
}

static int request_action(fighter_t* f, int id) { /* F:472-510 */
  if (is_action_end(f)) {
    set_current_action(f, id, 0);
    return 1;
  }
  if (f->action_id == id) return 0;
  const or_action_data* ad = action_data(f->action_id);
  if (ad->always_cancelable) {
    set_current_action(f, id, 0);
    return 1;
  }
  for (int c = 0; c < ad->n_cancel; c++) { /* GetCancelData: all matching windows, in order (AD:157-168) */
    const or_cancel_data* cd = &ad->cancel[c];
    if (!in_window(cd->s, cd->e, f->action_frame)) continue;
    int listed = 0;
    for (int k = 0; k < cd->n_ids; k++) listed |= (cd->ids[k] == id);
    if (listed) {
      if (cd->execute) {
        f->buffer_action_id = id;
        return 1;
      } else if (cd->buffer) {
        f->buffer_action_id = id;
      }
    }
  }
  return 0;
}

static int can_cancel_attack(const fighter_t* f) { /* F:531-539 */
  if (OR_CAN_CANCEL_ON_WHIFF) return 1;
  return f->hit_count > 0;
}

static int check_special_attack_input(const fighter_t* f) { /* F:569-583 */
  if (!is_attack_input(f->in_up[f->head])) return 0;
  for (int i = 1; i < OR_SPECIAL_ATTACK_HOLD_FRAME; i++)
    if (!is_attack_input(hist_in(f, i))) return 0;
  return 1;
}

static int check_forward_dash_input(const fighter_t* f) { /* F:585-609 */
  if (!is_forward_input(f, f->in_down[f->head])) return 0;
  for (int i = 1; i < OR_DASH_ALLOW_FRAME; i++) {
    if (is_backward_input(f, hist_in(f, i))) return 0;
    if (is_forward_input(f, hist_in(f, i))) {
      for (int j = i + 1; j < i + OR_DASH_ALLOW_FRAME; j++)
        if (!is_forward_input(f, hist_in(f, j)) && !is_backward_input(f, hist_in(f, j))) return 1;
      return 0;
    }
  }
  return 0;
}

static int check_backward_dash_input(const fighter_t* f) { /* F:611-635 */
  if (!is_backward_input(f, f->in_down[f->head])) return 0;
  for (int i = 1; i < OR_DASH_ALLOW_FRAME; i++) {
    if (is_forward_input(f, hist_in(f, i))) return 0;
    if (is_backward_input(f, hist_in(f, i))) {
      for (int j = i + 1; j < i + OR_DASH_ALLOW_FRAME; j++)
        if (!is_forward_input(f, hist_in(f, j)) && !is_backward_input(f, hist_in(f, j))) return 1;
      return 0;
    }
  }
  return 0;
}

static void update_action_request(fighter_t* f) { /* F:201-286 */
  if (f->has_won) {
    request_action(f, WIN);
    return;
  }
  if (f->reserve_damage_action_id != -1 && f->hitstun <= 0) {
    set_current_action(f, f->reserve_damage_action_id, 0);
    f->reserve_damage_action_id = -1;
    return;
  }
  if (f->buffer_action_id != -1 && can_cancel_attack(f) && f->hitstun <= 0) {
    set_current_action(f, f->buffer_action_id, 0);
    f->buffer_action_id = -1;
    return;
  }
  int in0 = f->in[f->head];
  int is_forward = is_forward_input(f, in0);
  int is_backward = is_backward_input(f, in0);
  int is_attack = is_attack_input(f->in_down[f->head]);
  if (check_special_attack_input(f)) {
    if (is_backward || is_forward)
      request_action(f, B_SPECIAL);
    else
      request_action(f, N_SPECIAL);
  } else if (is_attack) {
    if ((f->action_id == N_ATTACK || f->action_id == B_ATTACK) && !is_action_end(f))
      request_action(f, N_SPECIAL);
    else if (is_backward || is_forward)
      request_action(f, B_ATTACK);
    else
      request_action(f, N_ATTACK);
  }
  if (check_forward_dash_input(f))
    request_action(f, DASH_FORWARD);
  else if (check_backward_dash_input(f))
    request_action(f, DASH_BACKWARD);

  f->is_input_backward = is_backward;
  if (is_forward && is_backward)
    request_action(f, STAND);
  else if (is_forward)
    request_action(f, FORWARD);
  else if (is_backward) {
    if (f->is_reserve_proximity_guard)
      request_action(f, GUARD_PROXIMITY);
    else
      request_action(f, BACKWARD);
  } else
    request_action(f, STAND);
  f->is_reserve_proximity_guard = 0;
}

static void update_intro_action(fighter_t* f) { request_action(f, STAND); } /* F:193-196 */

static void update_movement(fighter_t* f, int fm) { /* F:291-319 */
  if (f->hitstun > 0) return;
  int sign = f->is_face_right ? 1 : -1;
  if (f->action_id == FORWARD) {
    f->pos_x = pos_plus_vel(fm, f->pos_x, OR_FORWARD_MOVE_SPEED, sign);
    return;
  } else if (f->action_id == BACKWARD) {
    f->pos_x = pos_minus_vel(fm, f->pos_x, OR_BACKWARD_MOVE_SPEED, sign);
    return;
  }
  const or_action_data* ad = action_data(f->action_id);
  for (int i = 0; i < ad->n_move; i++) { /* GetMovementData: first match (AD:146-155) */
    if (in_window(ad->move[i].s, ad->move[i].e, f->action_frame)) {
      f->velocity_x = ad->move[i].velocity_x;
      if (f->velocity_x != 0) f->pos_x = pos_plus_vel(fm, f->pos_x, f->velocity_x, sign);
      break;
    }
  }
}

static rect_t transform_to_fight_rect(int fm, const float r[4], float px, float py, int face_right) { /* F:706-719 */
  int sign = face_right ? 1 : -1;
  rect_t o;
  o.x = x_plus_rel(fm, px, r[0], sign);
  o.y = fadd(fm, py, r[1]);
  o.w = r[2];
  o.h = r[3];
  return o;
}

static void update_boxes(fighter_t* f, int fm) { /* ApplyCurrentActionData, F:671-697 */
  const or_action_data* ad = action_data(f->action_id);
  int fr = f->action_frame;
  f->n_hitboxes = 0;
  f->n_hurtboxes = 0;
  for (int i = 0; i < ad->n_hit; i++) {
    const or_hitbox_data* h = &ad->hit[i];
    if (!in_window(h->s, h->e, fr)) continue;
    float r[4] = {h->x, h->y, h->w, h->h};
    hitbox_t* b = &f->hitboxes[f->n_hitboxes++];
    b->rect = transform_to_fight_rect(fm, r, f->pos_x, f->pos_y, f->is_face_right);
    b->proximity = h->proximity;
    b->attack_id = h->attack_id;
  }
  for (int i = 0; i < ad->n_hurt; i++) {
    const or_box_data* h = &ad->hurt[i];
    if (!in_window(h->s, h->e, fr)) continue;
    float r[4] = {h->x, h->y, h->w, h->h};
    const float* rr = h->use_base ? OR_BASE_HURTBOX : r;
    f->hurtboxes[f->n_hurtboxes++] = transform_to_fight_rect(fm, rr, f->pos_x, f->pos_y, f->is_face_right);
  }
  const or_box_data* pb = 0;
  for (int i = 0; i < ad->n_push; i++) /* GetPushboxData: first match */
    if (in_window(ad->push[i].s, ad->push[i].e, fr)) {
      pb = &ad->push[i];
      break;
    }
  if (!pb) abort(); /* NullReferenceException in the reference (F:695) */
  float r[4] = {pb->x, pb->y, pb->w, pb->h};
  f->pushbox = transform_to_fight_rect(fm, pb->use_base ? OR_BASE_PUSHBOX : r, f->pos_x, f->pos_y, f->is_face_right);
}

static void apply_position_change(fighter_t* f, int fm, float x, float y) { /* F:331-350 */
  f->pos_x = fadd(fm, f->pos_x, x);
  f->pos_y = fadd(fm, f->pos_y, y);
  for (int i = 0; i < f->n_hitboxes; i++) {
    f->hitboxes[i].rect.x = fadd(fm, f->hitboxes[i].rect.x, x);
    f->hitboxes[i].rect.y = fadd(fm, f->hitboxes[i].rect.y, y);
  }
  for (int i = 0; i < f->n_hurtboxes; i++) {
    f->hurtboxes[i].x = fadd(fm, f->hurtboxes[i].x, x);
    f->hurtboxes[i].y = fadd(fm, f->hurtboxes[i].y, y);
  }
  f->pushbox.x = fadd(fm, f->pushbox.x, x);
  f->pushbox.y = fadd(fm, f->pushbox.y, y);
}

/* BoxBase (F:8-26): x is the centre */
static float bb_xmin(int fm, const rect_t* r) {
  if (fm == FS_FLOAT_DOUBLE) return (float)((double)r->x - (double)r->w / 2);
  return r->x - r->w / 2;
}
static float bb_xmax(int fm, const rect_t* r) {
  if (fm == FS_FLOAT_DOUBLE) return (float)((double)r->x + (double)r->w / 2);
  return r->x + r->w / 2;
}
static float bb_ymin(const rect_t* r) { return r->y; }
static float bb_ymax(int fm, const rect_t* r) { return fadd(fm, r->y, r->h); }
static int bb_overlaps(int fm, const rect_t* self, const rect_t* other) {
  int c1 = bb_xmax(fm, other) >= bb_xmin(fm, self);
  int c2 = bb_xmin(fm, other) <= bb_xmax(fm, self);
  int c3 = bb_ymax(fm, other) >= bb_ymin(self);
  int c4 = bb_ymin(other) <= bb_ymax(fm, self);
  return c1 && c2 && c3 && c4;
}

/* UnityEngine.Rect (engine): xMin = x, xMax = width + x; Overlaps is strict */
static float rect_xmax(int fm, const rect_t* r) { return fadd(fm, r->w, r->x); }
static float rect_ymax(int fm, const rect_t* r) { return fadd(fm, r->h, r->y); }
static int rect_overlaps(int fm, const rect_t* self, const rect_t* other) {
  return rect_xmax(fm, other) > self->x && other->x < rect_xmax(fm, self) && rect_ymax(fm, other) > self->y &&
         other->y < rect_ymax(fm, self);
}

static int can_attack_hit(const fighter_t* f, int attack_id) { /* F:408-420 */
  const or_attack_data* a = attack_data(attack_id);
  if (!a) return 1;
  if (f->hit_count >= a->number_of_hit) return 0;
  return 1;
}

static int notify_damaged(fighter_t* f, const or_attack_data* a) { /* F:357-398 */
  int is_guard_break = 0;
  if (a->guard_damage > 0) {
    f->guard -= a->guard_damage;
    if (f->guard < 0) {
      is_guard_break = 1;
      f->guard = 0;
    }
  }
  if (f->action_id == BACKWARD || action_data(f->action_id)->type == TYPE_GUARD) {
    if (is_guard_break) {
      set_current_action(f, a->guard_action, 0);
      f->reserve_damage_action_id = GUARD_BREAK;
      return DR_GUARD_BREAK;
    } else {
      set_current_action(f, a->guard_action, 0);
      return DR_GUARD;
    }
  } else {
    if (a->vital_damage > 0) {
      f->vital -= a->vital_damage;
      if (f->vital <= 0) f->vital = 0;
    }
    set_current_action(f, a->damage_action, 0);
    return DR_DAMAGE;
  }
}

static int get_hit_stun_frame(int result, const or_attack_data* a) { /* F:446-454 */
  if (result == DR_GUARD) return a->guard_stun;
  if (result == DR_GUARD_BREAK) return a->guard_break_stun;
  return a->hit_stun;
}

static void set_sprite_shake_frame(fighter_t* f, int frames) { /* F:438-444 (cosmetic) */
  if (frames > 6) frames = 6;
  f->sprite_shake = frames * (f->is_face_right ? -1 : 1);
}

/* ------------------------------------------------------------------------ */
/* BattleAI (AI:10-403), P2 only (isPlayer1 = false)                          */
/* ------------------------------------------------------------------------ */
enum { MP_NEUTRAL, MP_FAR1, MP_FAR2, MP_MID1, MP_MID2, MP_FALLBACK1, MP_FALLBACK2 };
enum { AP_NONE, AP_ONE_HIT, AP_TWO_HIT, AP_IMMEDIATE_SPECIAL, AP_DELAY_SPECIAL };

static void q_clear(queue_t* q) { q->head = q->count = 0; }
static void q_push(queue_t* q, int v) {
  q->q[(q->head + q->count) % 128] = v;
  q->count++;
}
static int q_pop(queue_t* q) {
  int v = q->q[q->head];
  q->head = (q->head + 1) % 128;
  q->count--;
  return v;
}

/* GetForwardInput / GetBackwardInput (AI:380-388): P1's bot (isPlayer1) walks Right */
static int bot_forward(int k) { return k == 0 ? IN_RIGHT : IN_LEFT; }
static int bot_backward(int k) { return k == 0 ? IN_LEFT : IN_RIGHT; }

static void add_forward(bot_t* b, int k, int n) { for (int i = 0; i < n; i++) q_push(&b->move_q, bot_forward(k)); }
static void add_backward(bot_t* b, int k, int n) { for (int i = 0; i < n; i++) q_push(&b->move_q, bot_backward(k)); }
static void add_forward_dash(bot_t* b, int k) { /* AI:330-335 */
  q_push(&b->move_q, bot_forward(k));
  q_push(&b->move_q, 0);
  q_push(&b->move_q, bot_forward(k));
}
static void add_backward_dash(bot_t* b, int k) { /* AI:337-342: enqueues *forward* inputs (reference quirk) */
  q_push(&b->move_q, bot_forward(k));
  q_push(&b->move_q, 0);
  q_push(&b->move_q, bot_forward(k));
}

static void set_move_plan(bot_t* b, int k, int plan) {
  switch (plan) {
    case MP_NEUTRAL: for (int i = 0; i < 30; i++) q_push(&b->move_q, 0); break;           /* AI:192-200 */
    case MP_FAR1: add_forward(b, k, 40); add_backward(b, k, 10); add_forward(b, k, 30); add_backward(b, k, 10); break;
    case MP_FAR2: add_forward_dash(b, k); add_backward(b, k, 25); add_forward_dash(b, k); add_backward(b, k, 25); break;
    case MP_MID1: add_forward(b, k, 30); add_backward(b, k, 10); add_forward(b, k, 20); add_backward(b, k, 10); break;
    case MP_MID2: add_forward_dash(b, k); add_backward(b, k, 30); break;
    case MP_FALLBACK1: add_backward(b, k, 60); break;
    case MP_FALLBACK2: add_backward_dash(b, k); add_backward(b, k, 60); break;
  }
  b->move_plan = plan;
  b->move_len = b->move_q.count;
}

static void set_attack_plan(bot_t* b, int plan) {
  queue_t* q = &b->attack_q;
  switch (plan) {
    case AP_NONE: for (int i = 0; i < 30; i++) q_push(q, 0); break; /* AI:255-263 */
    case AP_ONE_HIT: /* AI:265-274 */
      q_push(q, IN_ATTACK);
      for (int i = 0; i < 18; i++) q_push(q, 0);
      break;
    case AP_TWO_HIT: /* AI:276-290 */
      q_push(q, IN_ATTACK);
      for (int i = 0; i < 3; i++) q_push(q, 0);
      q_push(q, IN_ATTACK);
      for (int i = 0; i < 18; i++) q_push(q, 0);
      break;
    case AP_IMMEDIATE_SPECIAL: /* AI:292-301 */
      for (int i = 0; i < 60; i++) q_push(q, IN_ATTACK);
      q_push(q, 0);
      break;
    case AP_DELAY_SPECIAL: /* AI:303-312 */
      for (int i = 0; i < 120; i++) q_push(q, IN_ATTACK);
      q_push(q, 0);
      break;
  }
  b->attack_plan = plan;
  b->attack_len = q->count;
}

static void select_movement(arena_t* A, int k, const fight_state_t* s) { /* AI:68-126 */
  bot_t* b = &A->bot[k];
  if (s->distance_x > 4.0f) {
    int r = rng_range(A->rng, 0, 2);
    set_move_plan(b, k, r == 0 ? MP_FAR1 : MP_FAR2);
  } else if (s->distance_x > 3.0f) {
    int r = rng_range(A->rng, 0, 7);
    if (r <= 1) set_move_plan(b, k, MP_MID1);
    else if (r <= 3) set_move_plan(b, k, MP_MID2);
    else if (r == 4) set_move_plan(b, k, MP_FAR1);
    else if (r == 5) set_move_plan(b, k, MP_FAR2);
    else set_move_plan(b, k, MP_NEUTRAL);
  } else if (s->distance_x > 2.5f) {
    int r = rng_range(A->rng, 0, 5);
    if (r == 0) set_move_plan(b, k, MP_MID1);
    else if (r == 1) set_move_plan(b, k, MP_MID2);
    else if (r == 2) set_move_plan(b, k, MP_FALLBACK1);
    else if (r == 3) set_move_plan(b, k, MP_FALLBACK2);
    else set_move_plan(b, k, MP_NEUTRAL);
  } else if (s->distance_x > 2.0f) {
    int r = rng_range(A->rng, 0, 4);
    if (r == 0) set_move_plan(b, k, MP_FALLBACK1);
    else if (r == 1) set_move_plan(b, k, MP_FALLBACK2);
    else set_move_plan(b, k, MP_NEUTRAL);
  } else {
    int r = rng_range(A->rng, 0, 3);
    if (r == 0) set_move_plan(b, k, MP_FALLBACK1);
    else if (r == 1) set_move_plan(b, k, MP_FALLBACK2);
    else set_move_plan(b, k, MP_NEUTRAL);
  }
}

static void select_attack(arena_t* A, int k, const fight_state_t* s) { /* AI:128-190 */
  bot_t* b = &A->bot[k];
  if (s->opp_damage || s->opp_guard_break || s->opp_special_attack) {
    set_attack_plan(b, AP_TWO_HIT);
  } else if (s->distance_x > 4.0f) {
    int r = rng_range(A->rng, 0, 4);
    if (r <= 3) set_attack_plan(b, AP_NONE);
    else set_attack_plan(b, AP_DELAY_SPECIAL);
  } else if (s->distance_x > 3.0f) {
    if (s->opp_normal_attack) {
      set_attack_plan(b, AP_TWO_HIT);
      return;
    }
    int r = rng_range(A->rng, 0, 5);
    if (r <= 1) set_attack_plan(b, AP_NONE);
    else if (r <= 3) set_attack_plan(b, AP_ONE_HIT);
    else set_attack_plan(b, AP_DELAY_SPECIAL);
  } else if (s->distance_x > 2.5f) {
    int r = rng_range(A->rng, 0, 3);
    if (r == 0) set_attack_plan(b, AP_NONE);
    else if (r == 1) set_attack_plan(b, AP_ONE_HIT);
    else set_attack_plan(b, AP_TWO_HIT);
  } else if (s->distance_x > 2.0f) {
    int r = rng_range(A->rng, 0, 6);
    if (r <= 1) set_attack_plan(b, AP_ONE_HIT);
    else if (r <= 3) set_attack_plan(b, AP_TWO_HIT);
    else if (r == 4) set_attack_plan(b, AP_IMMEDIATE_SPECIAL);
    else set_attack_plan(b, AP_DELAY_SPECIAL);
  } else {
    int r = rng_range(A->rng, 0, 3);
    if (r == 0) set_attack_plan(b, AP_ONE_HIT);
    else set_attack_plan(b, AP_TWO_HIT);
  }
}

/* the bot of fighter k (0 = P1, isPlayer1; 1 = P2); its opponent is the other fighter (AI:34-39) */
static void bot_update_fight_state(arena_t* A, int k, int fm) { /* AI:344-363 */
  const fighter_t* opp = &A->f[1 - k];
  fight_state_t cur;
  memset(&cur, 0, sizeof cur);
  cur.valid = 1;
  /* GetDistanceX: Mathf.Abs(f2.x - f1.x) (AI:370-373) */
  cur.distance_x = fabsf(fsub(fm, A->f[1].pos_x, A->f[0].pos_x));
  cur.opp_damage = opp->action_id == DAMAGE;
  cur.opp_guard_break = opp->action_id == GUARD_BREAK;
  cur.opp_blocking = opp->action_id == GUARD_CROUCH || opp->action_id == GUARD_STAND || opp->action_id == GUARD_M;
  cur.opp_normal_attack = opp->action_id == N_ATTACK || opp->action_id == B_ATTACK;
  cur.opp_special_attack = opp->action_id == N_SPECIAL || opp->action_id == B_SPECIAL;
  cur.opp_action = opp->action_id;
  /* the reference's ascending copy loop: every slot 1..9 ends up equal to the old slot 0 */
  for (int i = 1; i < 10; i++) A->bot[k].fs[i] = A->bot[k].fs[i - 1];
  A->bot[k].fs[0] = cur;
}

static void bot_reset(arena_t* A, int k, int fm) { /* AI:393-403 */
  bot_t* b = &A->bot[k];
  q_clear(&b->move_q);
  q_clear(&b->attack_q);
  b->move_plan = b->attack_plan = -1;
  b->move_len = b->attack_len = 0;
  bot_update_fight_state(A, k, fm);
  for (int i = 0; i < 10; i++) b->fs[i] = b->fs[0];
}

static int bot_get_next_input(arena_t* A, int k, int fm) { /* AI:41-66 */
  int input = 0;
  bot_t* b = &A->bot[k];
  bot_update_fight_state(A, k, fm);
  const fight_state_t* s = &b->fs[5]; /* fightStateReadIndex (AI:32); null until a second call or a Reset */
  if (s->valid) {
    if (b->move_q.count > 0) input |= q_pop(&b->move_q);
    else select_movement(A, k, s);
    if (b->attack_q.count > 0) input |= q_pop(&b->attack_q);
    else select_attack(A, k, s);
  }
  return input;
}

/* ------------------------------------------------------------------------ */
/* BattleCore (BC:11-686)                                                    */
/* ------------------------------------------------------------------------ */
static void record_input(arena_t* A, int p1, int p2) { /* BC:593-607 */
  if (A->rec_idx >= OR_MAX_RECORDING_INPUT_FRAME) return;
  A->rec_last[0] = p1;
  A->rec_last[1] = p2;
  A->rec_idx++;
}

static fs_env_state get_environment_state(const arena_t* A) { /* BC:449-468 */
  fs_env_state s;
  s.p1Vital = A->f[0].vital;
  s.p2Vital = A->f[1].vital;
  s.p1Guard = A->f[0].guard;
  s.p2Guard = A->f[1].guard;
  s.p1Move = A->f[0].action_id;
  s.p1MoveFrame = A->f[0].action_frame;
  s.p2Move = A->f[1].action_id;
  s.p2MoveFrame = A->f[1].action_frame;
  s.p1Position = A->f[0].pos_x;
  s.p2Position = A->f[1].pos_x;
  s.globalFrame = A->frame_count;
  s.p1MostRecentAction = A->rec_idx > 0 ? A->rec_last[0] : 0;
  s.p2MostRecentAction = A->rec_idx > 0 ? A->rec_last[1] : 0;
  s.p1Hitstun = A->f[0].hitstun;
  s.p2Hitstun = A->f[1].hitstun;
  return s;
}

static void push_character_vs_character(arena_t* A, int fm) { /* BC:483-501 */
  rect_t r1 = A->f[0].pushbox, r2 = A->f[1].pushbox; /* Rect is a struct: copies */
  if (rect_overlaps(fm, &r1, &r2)) {
    if (A->f[0].pos_x < A->f[1].pos_x) {
      float d;
      if (fm == FS_FLOAT_DOUBLE) {
        double dd = (double)rect_xmax(fm, &r1) - (double)r2.x;
        apply_position_change(&A->f[0], fm, (float)(dd * -1 / 2), A->f[0].pos_y);
        apply_position_change(&A->f[1], fm, (float)(dd * 1 / 2), A->f[1].pos_y);
      } else {
        d = rect_xmax(fm, &r1) - r2.x;
        apply_position_change(&A->f[0], fm, d * -1 / 2, A->f[0].pos_y);
        apply_position_change(&A->f[1], fm, d * 1 / 2, A->f[1].pos_y);
      }
    } else if (A->f[0].pos_x > A->f[1].pos_x) {
      float d;
      if (fm == FS_FLOAT_DOUBLE) {
        double dd = (double)rect_xmax(fm, &r2) - (double)r1.x;
        apply_position_change(&A->f[0], fm, (float)(dd * 1 / 2), A->f[0].pos_y);
        apply_position_change(&A->f[1], fm, (float)(dd * -1 / 2), A->f[0].pos_y);
      } else {
        d = rect_xmax(fm, &r2) - r1.x;
        apply_position_change(&A->f[0], fm, d * 1 / 2, A->f[0].pos_y);
        apply_position_change(&A->f[1], fm, d * -1 / 2, A->f[0].pos_y);
      }
    }
  }
}

static void push_character_vs_background(arena_t* A, int fm) { /* BC:503-519 */
  const float stage_min = OR_BATTLE_AREA_WIDTH * -1 / 2;
  const float stage_max = OR_BATTLE_AREA_WIDTH / 2;
  for (int i = 0; i < 2; i++) {
    fighter_t* f = &A->f[i];
    if (bb_xmin(fm, &f->pushbox) < stage_min) {
      float dx = fm == FS_FLOAT_DOUBLE ? (float)((double)stage_min - (double)bb_xmin(fm, &f->pushbox))
                                       : stage_min - bb_xmin(fm, &f->pushbox);
      apply_position_change(f, fm, dx, f->pos_y);
    } else if (bb_xmax(fm, &f->pushbox) > stage_max) {
      float dx = fm == FS_FLOAT_DOUBLE ? (float)((double)stage_max - (double)bb_xmax(fm, &f->pushbox))
                                       : stage_max - bb_xmax(fm, &f->pushbox);
      apply_position_change(f, fm, dx, f->pos_y);
    }
  }
}

static void hitbox_hurtbox_collision(arena_t* A, int fm) { /* BC:521-591 */
  for (int ai = 0; ai < 2; ai++) {
    fighter_t* attacker = &A->f[ai];
    int is_hit = 0, is_proximity = 0, hit_attack_id = 0;
    for (int di = 0; di < 2; di++) {
      if (di == ai) continue;
      fighter_t* damaged = &A->f[di];
      for (int h = 0; h < attacker->n_hitboxes; h++) {
        const hitbox_t* hb = &attacker->hitboxes[h];
        if (!can_attack_hit(attacker, hb->attack_id)) continue;
        for (int u = 0; u < damaged->n_hurtboxes; u++) {
          if (bb_overlaps(fm, &hb->rect, &damaged->hurtboxes[u])) {
            if (hb->proximity) {
              is_proximity = 1;
            } else {
              is_hit = 1;
              hit_attack_id = hb->attack_id;
              break;
            }
          }
        }
        if (is_hit) break;
      }
      if (is_hit) {
        attacker->hit_count++; /* NotifyAttackHit, F:352-355 */
        const or_attack_data* ad = attack_data(hit_attack_id);
        int result = notify_damaged(damaged, ad);
        int stun = get_hit_stun_frame(result, attack_data(hit_attack_id));
        attacker->hitstun = stun;
        damaged->hitstun = stun;
        set_sprite_shake_frame(damaged, stun / 3);
      } else if (is_proximity) {
        if (damaged->is_input_backward) damaged->is_reserve_proximity_guard = 1; /* F:400-406 */
      }
    }
  }
}

/* TrainingManager.p1Input / p2Input (TrainingManager.cs:79-87): the current actor's GetInput() --
   the bot's last answer, or the remote actor's last received action (0 for an idle P2) */
static int get_input(const or_ctx* C, const arena_t* A, int k) {
  if (k == 0) return C->cfg.p1_mode == FS_P1_BOT ? A->bot_in[0] : A->actor_in[0];
  if (A->p2_bot) return A->bot_in[1];
  return C->cfg.p2_mode == FS_P2_NOOP ? 0 : A->actor_in[1];
}

static void update_intro_state(const or_ctx* C, arena_t* A, int fm) { /* BC:329-345 */
  int p1 = get_input(C, A, 0), p2 = get_input(C, A, 1);
  record_input(A, p1, p2);
  update_input(&A->f[0], p1);
  update_input(&A->f[1], p2);
  for (int i = 0; i < 2; i++) increment_action_frame(&A->f[i]);
  for (int i = 0; i < 2; i++) update_intro_action(&A->f[i]);
  for (int i = 0; i < 2; i++) update_movement(&A->f[i], fm);
  for (int i = 0; i < 2; i++) update_boxes(&A->f[i], fm);
  push_character_vs_character(A, fm);
  push_character_vs_background(A, fm);
}

static void update_fight_state(const or_ctx* C, arena_t* A, int fm) { /* BC:347-364 */
  int p1 = get_input(C, A, 0), p2 = get_input(C, A, 1);
  record_input(A, p1, p2);
  update_input(&A->f[0], p1);
  update_input(&A->f[1], p2);
  for (int i = 0; i < 2; i++) increment_action_frame(&A->f[i]);
  for (int i = 0; i < 2; i++) update_action_request(&A->f[i]);
  for (int i = 0; i < 2; i++) update_movement(&A->f[i], fm);
  for (int i = 0; i < 2; i++) update_boxes(&A->f[i], fm);
  push_character_vs_character(A, fm);
  push_character_vs_background(A, fm);
  hitbox_hurtbox_collision(A, fm);
}

static void update_end_state(arena_t* A, int fm) { /* BC:371-381 */
  for (int i = 0; i < 2; i++) increment_action_frame(&A->f[i]);
  for (int i = 0; i < 2; i++) update_action_request(&A->f[i]);
  for (int i = 0; i < 2; i++) update_movement(&A->f[i], fm);
  for (int i = 0; i < 2; i++) update_boxes(&A->f[i], fm);
  push_character_vs_character(A, fm);
  push_character_vs_background(A, fm);
}

/* TrainingManager.Step (TrainingManager.cs:59-77): P1's actor, then P2's, request their next
 * input unless the battle is over.  A bot answers at once (RequestNextInput -> getNextAIInput,
 * TrainingBattleAIActor.cs:38-41), drawing from the game's one RNG in that order; a remote actor's
 * answer is the action the next step delivers (fe_step_arena). */
static void training_step(or_ctx* C, arena_t* A, int battle_over) {
  A->emitted = 1;
  A->emitted_battle_over = battle_over;
  A->emitted_state = get_environment_state(A);
  if (battle_over) return;
  if (C->cfg.p1_mode == FS_P1_BOT) A->bot_in[0] = bot_get_next_input(A, 0, C->cfg.float_mode);
  if (A->p2_bot) A->bot_in[1] = bot_get_next_input(A, 1, C->cfg.float_mode);
}

static void change_round_state(or_ctx* C, arena_t* A, int state) { /* BC:247-327 */
  int fm = C->cfg.float_mode;
  A->round_state = state;
  switch (state) {
    case RS_STOP: break;
    case RS_INTRO:
      setup_battle_start(&A->f[0], OR_P1_START_X, 1);
      setup_battle_start(&A->f[1], OR_P2_START_X, 0);
      A->timer = 0.0f; /* introStateTime = 0 in training (BC:124-127) */
      /* BC:274-277: only a TrainingBattleAIActor is Reset, through GameManager.botP1 / botP2.  P1's
         bot is wrapped in a spectator (by_example), so it never is; P2's is when the game was
         launched with --p2-bot.  A bot switched in by P2_BOT in a game launched with a remote P2
         finds botP2 null: the Intro throws there, after SetupBattleStart, and nothing else of this
         ChangeRoundState runs -- the bot keeps its queues and FightStates. */
      if (A->p2_bot && C->cfg.p2_mode == FS_P2_BOT) bot_reset(A, 1, fm);
      break;
    case RS_FIGHT:
      A->frame_count = -1;
      A->rec_idx = 0;
      training_step(C, A, 0);
      break;
    case RS_KO:
      A->timer = 0.0f;
      clear_input(&A->f[0]);
      clear_input(&A->f[1]);
      break;
    case RS_END: {
      A->timer = 0.0f;
      int d0 = A->f[0].vital <= 0, d1 = A->f[1].vital <= 0;
      if (d0 + d1 == 1) {
        if (d0) A->f[1].has_won = 1; /* RequestWinAction, F:461-464 */
        else A->f[0].has_won = 1;
      }
      break;
    }
  }
}

/* BattleCore.FixedUpdate (BC:138-245).  cmd: 0 none, 1 RESET. */
static void fixed_update(or_ctx* C, arena_t* A, int cmd) {
  int fm = C->cfg.float_mode;
  if (cmd == 1) change_round_state(C, A, RS_STOP);
  switch (A->round_state) {
    case RS_STOP:
      change_round_state(C, A, RS_INTRO);
      break;
    case RS_INTRO:
      update_intro_state(C, A, fm);
      A->timer -= OR_FIXED_DT;
      if (A->timer <= 0.0f) change_round_state(C, A, RS_FIGHT);
      break;
    case RS_FIGHT: {
      /* synced mode: the driver only calls this once the actions are in (TrainingManager.Ready) */
      A->frame_count++;
      update_fight_state(C, A, fm);
      int battle_over = A->f[0].vital <= 0 || A->f[1].vital <= 0;
      if (battle_over) change_round_state(C, A, RS_KO);
      training_step(C, A, battle_over);
      break;
    }
    case RS_KO:
      A->timer -= OR_FIXED_DT;
      if (A->timer <= 0.0f) change_round_state(C, A, RS_END);
      break;
    case RS_END:
      update_end_state(A, fm);
      A->timer -= OR_FIXED_DT;
      if (A->timer <= 0.0f) change_round_state(C, A, RS_STOP);
      break;
  }
}

/* run FixedUpdate ticks until the game emits a state (TrainingManager.Step) */
static fs_env_state run_until_emission(or_ctx* C, arena_t* A, int first_cmd) {
  A->emitted = 0;
  int cmd = first_cmd;
  int guard = 0;
  while (!A->emitted) {
    fixed_update(C, A, cmd);
    cmd = 0;
    if (++guard > 16) abort();
  }
  return A->emitted_state;
}

/* ------------------------------------------------------------------------ */
/* FootsiesEnv post-processing (FE:336-405, 482-570)                          */
/* ------------------------------------------------------------------------ */
static int move_frame_simple(int move, int frame) { /* FE:339-358 */
  return (move == STAND || move == FORWARD || move == BACKWARD) ? 0 : frame;
}
static int dead_win_to_stand(int move) { return (move == DEAD || move == WIN) ? STAND : move; } /* FE:538-549 */

typedef struct {
  uint8_t guard[2], move[2], action[2], hitstun[2];
  float move_frame[2], position[2];
  int32_t frame;
} obs_t;

static obs_t extract_obs_info(const fs_env_state* s) { /* _extract_obs + _extract_info (FE:336-380) */
  obs_t o;
  o.guard[0] = (uint8_t)s->p1Guard;
  o.guard[1] = (uint8_t)s->p2Guard;
  o.move[0] = (uint8_t)move_index(s->p1Move);
  o.move[1] = (uint8_t)move_index(s->p2Move);
  o.move_frame[0] = (float)move_frame_simple(s->p1Move, s->p1MoveFrame);
  o.move_frame[1] = (float)move_frame_simple(s->p2Move, s->p2MoveFrame);
  o.position[0] = s->p1Position;
  o.position[1] = s->p2Position;
  o.frame = s->globalFrame;
  o.action[0] = (uint8_t)s->p1MostRecentAction;
  o.action[1] = (uint8_t)s->p2MostRecentAction;
  o.hitstun[0] = (uint8_t)s->p1Hitstun;
  o.hitstun[1] = (uint8_t)s->p2Hitstun;
  return o;
}

static void write_obs(or_ctx* C, int i, const obs_t* o) {
  for (int k = 0; k < 2; k++) {
    C->guard[2 * i + k] = o->guard[k];
    C->move[2 * i + k] = o->move[k];
    C->move_frame[2 * i + k] = o->move_frame[k];
    C->position[2 * i + k] = o->position[k];
    C->action[2 * i + k] = o->action[k];
    C->hitstun[2 * i + k] = o->hitstun[k];
  }
  C->frame[i] = o->frame;
}
static void write_final_obs(or_ctx* C, int i, const obs_t* o) {
  for (int k = 0; k < 2; k++) {
    C->f_guard[2 * i + k] = o->guard[k];
    C->f_move[2 * i + k] = o->move[k];
    C->f_move_frame[2 * i + k] = o->move_frame[k];
    C->f_position[2 * i + k] = o->position[k];
    C->f_action[2 * i + k] = o->action[k];
    C->f_hitstun[2 * i + k] = o->hitstun[k];
  }
  C->f_frame[i] = o->frame;
}

/* FE.delayed_frame_queue, a deque(maxlen = frame_delay + 1) of raw states (FE:129-131) */
static void dq_clear(arena_t* A) { A->dq_head = A->dq_count = 0; }
static void dq_append(or_ctx* C, arena_t* A, const fs_env_state* s) {
  int cap = C->cfg.frame_delay + 1;
  if (A->dq_count == cap) { /* a full deque drops its oldest entry */
    A->dq_head = (A->dq_head + 1) % cap;
    A->dq_count--;
  }
  A->dq[(A->dq_head + A->dq_count) % cap] = *s;
  A->dq_count++;
}
static fs_env_state dq_popleft(or_ctx* C, arena_t* A) {
  fs_env_state s = A->dq[A->dq_head];
  A->dq_head = (A->dq_head + 1) % (C->cfg.frame_delay + 1);
  A->dq_count--;
  return s;
}

/* FootsiesEnv.reset body after the (optional) RESET: read states until frame -1 */
static void fe_reset_arena(or_ctx* C, int i, const uint64_t* seeds, int hard) {
  arena_t* A = &C->a[i];
  if (seeds) rng_init(A->rng, (int32_t)(uint32_t)seeds[i]); /* SEED (BC:170-173) */
  fs_env_state s = A->cur_state; /* already at state(-1) unless a burst or RESET follows */
  if (A->reset_pending) s = run_until_emission(C, A, 0); /* the KO -> End -> Stop -> Intro -> Fight burst */
  if (hard) s = run_until_emission(C, A, 1);             /* RESET: Stop -> Intro -> Fight */
  A->reset_pending = 0;
  A->cum_reward = 0.0;
  A->cur_state = s;
  A->has_terminated = 0;
  dq_clear(A); /* FE:493, 502-504: frame_delay copies of the first state */
  while (A->dq_count < C->cfg.frame_delay) dq_append(C, A, &s);
  obs_t o = extract_obs_info(&s);
  write_obs(C, i, &o);
  C->reward[i] = 0.0;
  C->terminated[i] = 0;
}

static void fe_step_arena(or_ctx* C, int i, int p1, int p2) {
  arena_t* A = &C->a[i];
  if (A->reset_pending) { /* FS_AUTORESET_NEXT_STEP: this step is the reset */
    fe_reset_arena(C, i, 0, 0);
    return;
  }
  /* the actions arrive; the synced game runs its Fight tick (TrainingRemoteActor.cs:93-117) */
  if (C->cfg.p1_mode != FS_P1_BOT) A->actor_in[0] = p1 & 7;                  /* by_example sends none (FE:522-523) */
  if (C->cfg.p2_mode == FS_P2_EXTERNAL && !A->p2_bot) A->actor_in[1] = p2 & 7; /* FE:525-527 */
  fs_env_state prev = A->cur_state;
  fs_env_state st = run_until_emission(C, A, 0);
  A->cur_state = st;
  dq_append(C, A, &st); /* FE:533-535: the newest state in, the oldest out */
  fs_env_state obs_state = dq_popleft(C, A);
  obs_state.p1Move = dead_win_to_stand(obs_state.p1Move);
  obs_state.p2Move = dead_win_to_stand(obs_state.p2Move);
  obs_t o = extract_obs_info(&obs_state);
  int terminated = st.p1Vital == 0 || st.p2Vital == 0;
  double reward;
  if (C->cfg.dense_reward) { /* FE:388-405 */
    reward = 0.0;
    if (st.p1Guard < prev.p1Guard) reward -= 0.3;
    if (st.p2Guard < prev.p2Guard) reward += 0.3;
    A->cum_reward += reward;
    if (terminated) reward += (double)(st.p2Vital == 0 ? 1 : -1) - A->cum_reward;
  } else { /* FE:382-386 */
    reward = terminated ? (st.p2Vital == 0 ? 1.0 : -1.0) : 0.0;
  }
  C->reward[i] = reward;
  C->terminated[i] = (uint8_t)terminated;
  A->has_terminated = terminated;
  if (terminated && C->cfg.autoreset_mode == FS_AUTORESET_SAME_STEP) {
    write_final_obs(C, i, &o);
    double r = C->reward[i];
    A->reset_pending = 1; /* Unity runs the KO -> ... -> Fight burst on its own (BC:212-243) */
    fe_reset_arena(C, i, 0, 0 /* FE.reset after a terminated step sends no RESET (FE:490-491) */);
    C->reward[i] = r;
    C->terminated[i] = 1;
  } else {
    write_obs(C, i, &o);
    if (terminated) A->reset_pending = 1;
  }
}

/* ------------------------------------------------------------------------ */
/* C API (mirrors include/footsies.h with host pointers)                     */
/* ------------------------------------------------------------------------ */
static void* xcalloc(size_t n, size_t s) {
  void* p = calloc(n ? n : 1, s);
  if (!p) abort();
  return p;
}

static void new_fighter(fighter_t* f) { /* `new Fighter()` (BC:93-94) field defaults */
  memset(f, 0, sizeof *f);
  f->buffer_action_id = -1;
  f->reserve_damage_action_id = -1;
}

OR_EXPORT int or_create(const fs_config* cfg, or_handle* out) {
  if (!cfg || !out || cfg->num_envs <= 0) return FS_E_INVALID;
  if (cfg->frame_delay < 0) return FS_E_INVALID;
  if (cfg->p2_mode < 0 || cfg->p2_mode > 2) return FS_E_INVALID;
  if (cfg->p1_mode != FS_P1_EXTERNAL && cfg->p1_mode != FS_P1_BOT) return FS_E_INVALID;
  or_ctx* C = (or_ctx*)xcalloc(1, sizeof(or_ctx));
  C->cfg = *cfg;
  int n = C->n = cfg->num_envs;
  C->a = (arena_t*)xcalloc((size_t)n, sizeof(arena_t));
  C->guard = xcalloc(2 * n, 1);
  C->move = xcalloc(2 * n, 1);
  C->action = xcalloc(2 * n, 1);
  C->hitstun = xcalloc(2 * n, 1);
  C->terminated = xcalloc(n, 1);
  C->truncated = xcalloc(n, 1);
  C->move_frame = xcalloc(2 * n, sizeof(float));
  C->position = xcalloc(2 * n, sizeof(float));
  C->reward = xcalloc(n, sizeof(double));
  C->frame = xcalloc(n, sizeof(int32_t));
  C->f_guard = xcalloc(2 * n, 1);
  C->f_move = xcalloc(2 * n, 1);
  C->f_action = xcalloc(2 * n, 1);
  C->f_hitstun = xcalloc(2 * n, 1);
  C->f_move_frame = xcalloc(2 * n, sizeof(float));
  C->f_position = xcalloc(2 * n, sizeof(float));
  C->f_frame = xcalloc(n, sizeof(int32_t));
#pragma omp parallel for schedule(static) if (C->n >= 1024)
  for (int i = 0; i < n; i++) {
    arena_t* A = &C->a[i];
    new_fighter(&A->f[0]);
    new_fighter(&A->f[1]);
    A->round_state = RS_STOP;
    A->bot[0].move_plan = A->bot[0].attack_plan = A->bot[1].move_plan = A->bot[1].attack_plan = -1;
    A->p2_bot = cfg->p2_mode == FS_P2_BOT; /* GameManager.cs:193 (--p2-bot) */
    rng_init(A->rng, (int32_t)(uint32_t)(cfg->base_seed + cfg->arena_base + (uint64_t)i));
    /* game start: Stop -> Intro -> Fight, state(-1) emitted */
    A->cur_state = run_until_emission(C, A, 0);
    A->has_terminated = 1; /* FE.__init__ (FE:191): the first reset() sends no RESET */
    A->dq = (fs_env_state*)xcalloc((size_t)cfg->frame_delay + 1, sizeof(fs_env_state));
    while (A->dq_count < cfg->frame_delay) dq_append(C, A, &A->cur_state);
    obs_t o = extract_obs_info(&A->cur_state);
    write_obs(C, i, &o);
  }
  *out = C;
  return FS_OK;
}

OR_EXPORT int or_reset(or_handle C, const uint64_t* seeds, const uint8_t* mask, int flags) {
  if (!C) return FS_E_INVALID;
#pragma omp parallel for schedule(static) if (C->n >= 1024)
  for (int i = 0; i < C->n; i++) {
    if (mask && !mask[i]) continue;
    if (flags == FS_RESET_SEED_ONLY) { /* SEED alone (BC:170-173) */
      if (seeds) rng_init(C->a[i].rng, (int32_t)(uint32_t)seeds[i]);
      continue;
    }
    int hard = (flags == FS_RESET_HARD) || !C->a[i].has_terminated;
    fe_reset_arena(C, i, seeds, hard);
  }
  return FS_OK;
}

/* P2_BOT (BC:158-167) on the masked arenas: P2's actor becomes the bot or the remote actor again */
OR_EXPORT int or_set_p2_mode(or_handle C, int mode, const uint8_t* mask) {
  if (!C || (mode != FS_P2_EXTERNAL && mode != FS_P2_BOT)) return FS_E_INVALID;
  if (C->cfg.p2_mode != FS_P2_EXTERNAL) return FS_E_UNSUPPORTED;
  for (int i = 0; i < C->n; i++)
    if (!mask || mask[i]) C->a[i].p2_bot = mode == FS_P2_BOT;
  return FS_OK;
}

OR_EXPORT int or_step(or_handle C, const uint8_t* p1, const uint8_t* p2) {
  if (!C || (!p1 && C->cfg.p1_mode != FS_P1_BOT)) return FS_E_INVALID;
  if (C->cfg.p2_mode == FS_P2_EXTERNAL && !p2) return FS_E_INVALID;
#pragma omp parallel for schedule(static) if (C->n >= 1024)
  for (int i = 0; i < C->n; i++) fe_step_arena(C, i, p1 ? p1[i] : 0, p2 ? p2[i] : 0);
  C->steps++;
  return FS_OK;
}

/* fs_step_masked: only arenas with active[i] != 0 run FootsiesEnv.step; the others are
   separate environments that were not stepped (state and outputs untouched) */
OR_EXPORT int or_step_masked(or_handle C, const uint8_t* p1, const uint8_t* p2, const uint8_t* active) {
  if (!C || (!p1 && C->cfg.p1_mode != FS_P1_BOT) || !active) return FS_E_INVALID;
  if (C->cfg.p2_mode == FS_P2_EXTERNAL && !p2) return FS_E_INVALID;
#pragma omp parallel for schedule(static) if (C->n >= 1024)
  for (int i = 0; i < C->n; i++)  /* (each arena's delayed-frame queue advances with its own steps) */
    if (active[i]) fe_step_arena(C, i, p1 ? p1[i] : 0, p2 ? p2[i] : 0);
  C->steps++;
  return FS_OK;
}

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
/* the synthetic action stream of BASELINE.md / SURVEY.md §8(d) */
OR_EXPORT uint8_t or_hash_action(uint64_t seed, uint64_t env, uint64_t t, int player) {
  return (uint8_t)(splitmix64(seed ^ (env * 0x9E3779B97F4A7C15ull) ^ ((t << 1) | (uint64_t)player)) & 7u);
}

/* n steps with hashed actions (throughput baseline); outputs of the last step remain */
OR_EXPORT int or_step_n_hashed(or_handle C, int n, uint64_t action_seed) {
  if (!C || n < 0) return FS_E_INVALID;
  uint64_t t0 = C->steps;
#pragma omp parallel for schedule(static) if (C->n >= 1024)
  for (int i = 0; i < C->n; i++)
    for (int k = 0; k < n; k++) {
      const uint64_t env = C->cfg.arena_base + (uint64_t)i;
      fe_step_arena(C, i, or_hash_action(action_seed, env, t0 + (uint64_t)k, 0),
                    or_hash_action(action_seed, env, t0 + (uint64_t)k, 1));
    }
  C->steps += (uint64_t)n;
  return FS_OK;
}

OR_EXPORT int or_outputs_get(or_handle C, fs_outputs* o) {
  if (!C || !o) return FS_E_INVALID;
  o->guard = C->guard;
  o->move = C->move;
  o->move_frame = C->move_frame;
  o->position = C->position;
  o->reward = C->reward;
  o->terminated = C->terminated;
  o->truncated = C->truncated;
  o->frame = C->frame;
  o->action = C->action;
  o->hitstun = C->hitstun;
  o->final_guard = C->f_guard;
  o->final_move = C->f_move;
  o->final_move_frame = C->f_move_frame;
  o->final_position = C->f_position;
  o->final_frame = C->f_frame;
  o->final_action = C->f_action;
  o->final_hitstun = C->f_hitstun;
  return FS_OK;
}

OR_EXPORT int or_get_env_state(or_handle C, fs_env_state* out) {
  if (!C || !out) return FS_E_INVALID;
  for (int i = 0; i < C->n; i++) out[i] = get_environment_state(&C->a[i]);
  return FS_OK;
}

/* a BattleAI in canonical form: queues as (plan, dequeued count), plan -1 = empty; the FightState
   its next call reads (fightStates[5] == slot 0 after the ascending copy, AI:358-361) */
static void bot_export(const bot_t* b, int32_t* mp, int32_t* mi, int32_t* ap, int32_t* ai, float* pd, int32_t* po,
                       uint8_t* ready) {
  *mp = b->move_q.count > 0 ? b->move_plan : -1;
  *mi = b->move_q.count > 0 ? b->move_len - b->move_q.count : 0;
  *ap = b->attack_q.count > 0 ? b->attack_plan : -1;
  *ai = b->attack_q.count > 0 ? b->attack_len - b->attack_q.count : 0;
  *pd = b->fs[0].valid ? b->fs[0].distance_x : 0.0f;
  *po = b->fs[0].valid ? b->fs[0].opp_action : STAND;
  *ready = (uint8_t)b->fs[0].valid;
}

OR_EXPORT int or_get_state(or_handle C, fs_arena_state* out) {
  if (!C || !out) return FS_E_INVALID;
  for (int i = 0; i < C->n; i++) {
    const arena_t* A = &C->a[i];
    fs_arena_state* s = &out[i];
    memset(s, 0, sizeof *s);
    for (int k = 0; k < 2; k++) {
      const fighter_t* f = &A->f[k];
      fs_fighter_state* g = &s->f[k];
      g->position_x = f->pos_x;
      g->action_id = f->action_id;
      g->action_frame = f->action_frame;
      g->hit_count = f->hit_count;
      g->hitstun = f->hitstun;
      g->vital = f->vital;
      g->guard = f->guard;
      g->buffer_action_id = f->buffer_action_id;
      g->reserve_action_id = f->reserve_damage_action_id;
      uint32_t h = 0;
      for (int j = 15; j >= 0; j--) h = (h << 2) | (uint32_t)(hist_in(f, j) & 3);
      g->input_dir_history = h;
      int hold = 0;
      while (hold < 63 && hold < OR_INPUT_RECORD_FRAME && (hist_in(f, hold) & IN_ATTACK)) hold++;
      g->attack_hold = hold;
      g->is_input_backward = (uint8_t)f->is_input_backward;
      g->is_reserve_proximity_guard = (uint8_t)f->is_reserve_proximity_guard;
      g->has_won = (uint8_t)f->has_won;
      g->facing_flipped = (uint8_t)(f->is_face_right != (k == 0)); /* SetupBattleStart: isFaceRight = isPlayerOne */
      g->position_y = f->pos_y;
    }
    s->frame_count = A->frame_count;
    s->recording_count = (int32_t)A->rec_idx;
    s->recording_last[0] = (uint8_t)A->rec_last[0];
    s->recording_last[1] = (uint8_t)A->rec_last[1];
    s->actor_input[0] = (uint8_t)A->actor_in[0];
    s->actor_input[1] = (uint8_t)A->actor_in[1];
    s->reset_pending = (uint8_t)A->reset_pending;
    s->has_terminated = (uint8_t)A->has_terminated;
    s->cumulative_reward = A->cum_reward;
    memcpy(s->rng, A->rng, sizeof s->rng);
    bot_export(&A->bot[1], &s->move_plan, &s->move_index, &s->attack_plan, &s->attack_index, &s->prev_distance,
               &s->prev_opponent_action, &s->bot_ready[1]);
    bot_export(&A->bot[0], &s->p1_move_plan, &s->p1_move_index, &s->p1_attack_plan, &s->p1_attack_index,
               &s->p1_prev_distance, &s->p1_prev_opponent_action, &s->bot_ready[0]);
    s->p2_bot = (uint8_t)A->p2_bot;
    s->bot_input[0] = (uint8_t)A->bot_in[0];
    s->bot_input[1] = (uint8_t)A->bot_in[1];
  }
  return FS_OK;
}

/* STATE_LOAD of the canonical state (fs_set_state).  The 180-deep histories are rebuilt
   from what fs_arena_state carries -- directions of input[0..15], Attack over the held run
   input[0..hold-1] -- with zeros beyond; inputDown / inputUp follow from input (F:182-184).
   Boxes and velocity_x are left for the next UpdateBoxes / UpdateMovement to set.  A
   pending terminal arena resumes in KO with its timer at 0 (BC:303-306).  With the scripted
   bot, its queues are rebuilt by enqueueing each plan (set_move_plan / set_attack_plan) and
   popping the inputs already consumed, and every FightState slot holds the previous call's
   state: getNextAIInput's ascending copy loop overwrites slots 1..9 with slot 0 before it
   reads slot 5 (AI:358-361), so slot 0 is all a later call can observe. */
static void bot_set_state(arena_t* A, int k, int32_t mp, int32_t mi, int32_t ap, int32_t ai, float pd, int32_t opp,
                          int ready) {
  bot_t* b = &A->bot[k];
  q_clear(&b->move_q);
  q_clear(&b->attack_q);
  b->move_plan = b->attack_plan = -1;
  b->move_len = b->attack_len = 0;
  if (mp >= 0) {
    set_move_plan(b, k, mp);
    for (int i = 0; i < mi && b->move_q.count > 0; i++) q_pop(&b->move_q);
  }
  if (ap >= 0) {
    set_attack_plan(b, ap);
    for (int i = 0; i < ai && b->attack_q.count > 0; i++) q_pop(&b->attack_q);
  }
  fight_state_t prev;
  memset(&prev, 0, sizeof prev);
  if (!ready) { /* fightStates all null: the next call answers 0 */
    for (int i = 0; i < 10; i++) b->fs[i] = prev;
    return;
  }
  prev.valid = 1;
  prev.distance_x = pd;
  prev.opp_damage = opp == DAMAGE;
  prev.opp_guard_break = opp == GUARD_BREAK;
  prev.opp_blocking = opp == GUARD_CROUCH || opp == GUARD_STAND || opp == GUARD_M;
  prev.opp_normal_attack = opp == N_ATTACK || opp == B_ATTACK;
  prev.opp_special_attack = opp == N_SPECIAL || opp == B_SPECIAL;
  prev.opp_action = opp;
  for (int i = 0; i < 10; i++) b->fs[i] = prev;
}

OR_EXPORT int or_set_state(or_handle C, const fs_arena_state* in) {
  if (!C || !in) return FS_E_INVALID;
  for (int i = 0; i < C->n; i++) {
    arena_t* A = &C->a[i];
    const fs_arena_state* s = &in[i];
    for (int k = 0; k < 2; k++) {
      fighter_t* f = &A->f[k];
      const fs_fighter_state* g = &s->f[k];
      f->pos_x = g->position_x; /* LoadState (F:741-744) */
      f->pos_y = g->position_y;
      f->is_face_right = (k == 0) != (g->facing_flipped != 0);
      f->action_id = g->action_id;
      f->action_frame = g->action_frame;
      f->hit_count = g->hit_count;
      f->hitstun = g->hitstun;
      f->vital = g->vital;
      f->guard = g->guard;
      f->buffer_action_id = g->buffer_action_id;
      f->reserve_damage_action_id = g->reserve_action_id;
      clear_input(f);
      f->head = 0;
      for (int j = 0; j < OR_INPUT_RECORD_FRAME; j++) {
        int v = j < 16 ? (int)((g->input_dir_history >> (2 * j)) & 3u) : 0;
        if (j < g->attack_hold) v |= IN_ATTACK;
        f->in[j] = v;
      }
      for (int j = 0; j < OR_INPUT_RECORD_FRAME; j++) {
        int next = j + 1 < OR_INPUT_RECORD_FRAME ? f->in[j + 1] : 0;
        f->in_down[j] = (f->in[j] ^ next) & f->in[j];
        f->in_up[j] = (f->in[j] ^ next) & ~f->in[j];
      }
      f->is_input_backward = g->is_input_backward;
      f->is_reserve_proximity_guard = g->is_reserve_proximity_guard;
      f->has_won = g->has_won;
    }
    A->frame_count = s->frame_count;
    A->rec_idx = (uint32_t)s->recording_count;
    A->rec_last[0] = s->recording_last[0];
    A->rec_last[1] = s->recording_last[1];
    A->actor_in[0] = s->actor_input[0];
    A->actor_in[1] = s->actor_input[1];
    A->bot_in[0] = s->bot_input[0];
    A->bot_in[1] = s->bot_input[1];
    A->p2_bot = s->p2_bot;
    A->reset_pending = s->reset_pending;
    A->has_terminated = s->has_terminated;
    A->cum_reward = s->cumulative_reward;
    A->round_state = s->reset_pending ? RS_KO : RS_FIGHT;
    A->timer = 0.0f;
    memcpy(A->rng, s->rng, sizeof A->rng);
    bot_set_state(A, 1, s->move_plan, s->move_index, s->attack_plan, s->attack_index, s->prev_distance,
                  s->prev_opponent_action, s->bot_ready[1]);
    bot_set_state(A, 0, s->p1_move_plan, s->p1_move_index, s->p1_attack_plan, s->p1_attack_index,
                  s->p1_prev_distance, s->p1_prev_opponent_action, s->bot_ready[0]);
    A->cur_state = get_environment_state(A);
  }
  return FS_OK;
}

OR_EXPORT void or_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}
OR_EXPORT int or_get_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

OR_EXPORT void or_destroy(or_handle C) {
  if (!C) return;
  for (int i = 0; i < C->n; i++) free(C->a[i].dq);
  free(C->a);
  free(C->guard); free(C->move); free(C->action); free(C->hitstun); free(C->terminated); free(C->truncated);
  free(C->move_frame); free(C->position); free(C->reward); free(C->frame);
  free(C->f_guard); free(C->f_move); free(C->f_action); free(C->f_hitstun);
  free(C->f_move_frame); free(C->f_position); free(C->f_frame);
  free(C);
}
