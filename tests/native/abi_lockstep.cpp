// abi_lockstep.cpp -- a C++ consumer of include/footsies.h, built with host-side
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/native/Makefile) over a
// sanitizer build of libfootsies' host code, stepping the HIP path in lockstep with
// the CPU oracle (linked in: test infrastructure) and comparing the canonical state
// bitwise.  Also: determinism (two handles, same config, identical outputs), the
// packed gather records, and the error paths of the C-ABI.  Exit status 0 = pass.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "footsies.h"

extern "C" {
typedef void* or_handle;
int or_create(const fs_config* cfg, or_handle* out);
int or_reset(or_handle h, const uint64_t* seeds, const uint8_t* mask, int flags);
int or_step(or_handle h, const uint8_t* p1, const uint8_t* p2);
int or_step_n_hashed(or_handle h, int n, uint64_t action_seed);
int or_get_state(or_handle h, fs_arena_state* out);
uint8_t or_hash_action(uint64_t seed, uint64_t env, uint64_t t, int player);
void or_set_threads(int n);
void or_destroy(or_handle h);
}

static int failures = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fprintf(stderr, "\n");                           \
      failures++;                                      \
    }                                                  \
  } while (0)

static bool same_fighter(const fs_fighter_state& a, const fs_fighter_state& b) {
  return memcmp(&a.position_x, &b.position_x, 4) == 0 && a.action_id == b.action_id &&
         a.action_frame == b.action_frame && a.hit_count == b.hit_count && a.hitstun == b.hitstun &&
         a.vital == b.vital && a.guard == b.guard && a.buffer_action_id == b.buffer_action_id &&
         a.reserve_action_id == b.reserve_action_id && a.input_dir_history == b.input_dir_history &&
         a.attack_hold == b.attack_hold && a.is_input_backward == b.is_input_backward &&
         a.is_reserve_proximity_guard == b.is_reserve_proximity_guard && a.has_won == b.has_won &&
         a.facing_flipped == b.facing_flipped && memcmp(&a.position_y, &b.position_y, 4) == 0;
}
static bool same_arena(const fs_arena_state& a, const fs_arena_state& b, bool bot) {
  bool ok = same_fighter(a.f[0], b.f[0]) && same_fighter(a.f[1], b.f[1]) && a.frame_count == b.frame_count &&
            a.recording_count == b.recording_count && memcmp(a.recording_last, b.recording_last, 2) == 0 &&
            a.reset_pending == b.reset_pending && a.has_terminated == b.has_terminated &&
            memcmp(&a.cumulative_reward, &b.cumulative_reward, 8) == 0;
  if (bot)
    ok = ok && memcmp(a.rng, b.rng, 16) == 0 && a.move_plan == b.move_plan && a.move_index == b.move_index &&
         a.attack_plan == b.attack_plan && a.attack_index == b.attack_index &&
         memcmp(&a.prev_distance, &b.prev_distance, 4) == 0 && a.prev_opponent_action == b.prev_opponent_action;
  // the actors (ABI 2): the game RNG is kept in every mode, the P1 bot's fields likewise
  ok = ok && memcmp(a.rng, b.rng, 16) == 0 && memcmp(a.actor_input, b.actor_input, 2) == 0 &&
       a.p2_bot == b.p2_bot && memcmp(a.bot_ready, b.bot_ready, 2) == 0 && memcmp(a.bot_input, b.bot_input, 2) == 0 &&
       a.p1_move_plan == b.p1_move_plan && a.p1_move_index == b.p1_move_index &&
       a.p1_attack_plan == b.p1_attack_plan && a.p1_attack_index == b.p1_attack_index &&
       memcmp(&a.p1_prev_distance, &b.p1_prev_distance, 4) == 0 &&
       a.p1_prev_opponent_action == b.p1_prev_opponent_action;
  return ok;
}

static void compare_states(fs_handle h, or_handle o, int n, bool bot, const char* what) {
  std::vector<fs_arena_state> g(n), c(n);
  CHECK(fs_get_state(h, g.data()) == FS_OK, "fs_get_state: %s", fs_last_error(h));
  CHECK(or_get_state(o, c.data()) == 0, "or_get_state");
  int bad = 0, first = -1;
  for (int i = 0; i < n; i++)
    if (!same_arena(g[i], c[i], bot)) {
      if (first < 0) first = i;
      bad++;
    }
  CHECK(bad == 0, "%s: %d of %d arenas differ from the oracle (first %d)", what, bad, n, first);
}

static void lockstep(int p2_mode, int autoreset, int float_mode, int n, int steps, int fused) {
  fs_config cfg{};
  cfg.num_envs = n;
  cfg.device_id = 0;
  cfg.p2_mode = p2_mode;
  cfg.dense_reward = 1;
  cfg.float_mode = float_mode;
  cfg.autoreset_mode = autoreset;
  cfg.base_seed = 11;
  fs_handle h = nullptr;
  or_handle o = nullptr;
  CHECK(fs_create(&cfg, &h) == FS_OK, "fs_create: %s", fs_last_error(nullptr));
  fs_config ocfg = cfg;
  ocfg.device_id = -1;
  CHECK(or_create(&ocfg, &o) == 0, "or_create");
  if (!h || !o) {
    fs_destroy(h);
    if (o) or_destroy(o);
    return;
  }
  CHECK(fs_reset(h, nullptr, nullptr, FS_RESET_HARD) == FS_OK, "fs_reset");
  or_reset(o, nullptr, nullptr, FS_RESET_HARD);
  std::vector<uint8_t> p1(n), p2(n);
  const uint64_t seed = 0x5EED;
  for (int t = 0; t < steps; t++) {
    for (int i = 0; i < n; i++) {
      p1[i] = or_hash_action(seed, i, t, 0);
      p2[i] = or_hash_action(seed, i, t, 1);
    }
    CHECK(fs_step(h, p1.data(), p2.data(), FS_ACT_HOST) == FS_OK, "fs_step: %s", fs_last_error(h));
    or_step(o, p1.data(), p2_mode == FS_P2_EXTERNAL ? p2.data() : nullptr);
  }
  CHECK(fs_sync(h) == FS_OK, "fs_sync");
  compare_states(h, o, n, p2_mode == FS_P2_BOT, "after single steps");
  if (fused) {  // fs_step_n with in-kernel hashed actions continues the same counter
    CHECK(fs_step_n(h, fused, nullptr, nullptr, seed, nullptr) == FS_OK, "fs_step_n: %s", fs_last_error(h));
    or_step_n_hashed(o, fused, seed);
    CHECK(fs_steps_taken(h) == (uint64_t)(steps + fused), "fs_steps_taken");
    CHECK(fs_sync(h) == FS_OK, "fs_sync");
    compare_states(h, o, n, p2_mode == FS_P2_BOT, "after fused steps");
  }
  fs_destroy(h);
  or_destroy(o);
}

static void determinism_and_pack(int n) {
  fs_config cfg{};
  cfg.num_envs = n;
  cfg.p2_mode = FS_P2_BOT;
  cfg.dense_reward = 1;
  cfg.base_seed = 3;
  fs_handle a = nullptr, b = nullptr;
  CHECK(fs_create(&cfg, &a) == FS_OK && fs_create(&cfg, &b) == FS_OK, "fs_create");
  if (!a || !b) {
    fs_destroy(a);
    fs_destroy(b);
    return;
  }
  fs_reset(a, nullptr, nullptr, FS_RESET_HARD);
  fs_reset(b, nullptr, nullptr, FS_RESET_HARD);
  CHECK(fs_step_n(a, 500, nullptr, nullptr, 9, nullptr) == FS_OK, "fs_step_n a");
  CHECK(fs_step_n(b, 500, nullptr, nullptr, 9, nullptr) == FS_OK, "fs_step_n b");
  void *ra = nullptr, *rb = nullptr;
  CHECK(hipMalloc(&ra, (size_t)n * FS_RECORD_BYTES) == hipSuccess, "hipMalloc");
  CHECK(hipMalloc(&rb, (size_t)n * FS_RECORD_BYTES) == hipSuccess, "hipMalloc");
  CHECK(fs_pack_outputs(a, ra) == FS_OK && fs_pack_outputs(b, rb) == FS_OK, "fs_pack_outputs");
  fs_sync(a);
  fs_sync(b);
  std::vector<uint8_t> ha((size_t)n * FS_RECORD_BYTES), hb(ha.size());
  CHECK(hipMemcpy(ha.data(), ra, ha.size(), hipMemcpyDeviceToHost) == hipSuccess, "copy");
  CHECK(hipMemcpy(hb.data(), rb, hb.size(), hipMemcpyDeviceToHost) == hipSuccess, "copy");
  CHECK(ha == hb, "two handles with one config diverged");
  // the records hold the outputs: frame of arena i at bytes [28, 32)
  fs_outputs o{};
  fs_outputs_get(a, &o);
  std::vector<int32_t> frame(n);
  CHECK(hipMemcpy(frame.data(), o.frame, 4 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess, "copy frame");
  int bad = 0;
  for (int i = 0; i < n; i++) bad += memcmp(&ha[(size_t)i * FS_RECORD_BYTES + 28], &frame[i], 4) != 0;
  CHECK(bad == 0, "packed frame field differs for %d arenas", bad);
  (void)hipFree(ra);
  (void)hipFree(rb);
  fs_destroy(a);
  fs_destroy(b);
}

static void error_paths() {
  fs_config cfg{};
  fs_handle h = nullptr;
  cfg.num_envs = 0;
  CHECK(fs_create(&cfg, &h) == FS_E_INVALID && !h, "num_envs 0 accepted");
  CHECK(fs_last_error(nullptr) && fs_last_error(nullptr)[0], "no message for a failed fs_create");
  cfg.num_envs = 8;
  cfg.p2_mode = 7;
  CHECK(fs_create(&cfg, &h) == FS_E_INVALID && !h, "bad p2_mode accepted");
  cfg.p2_mode = FS_P2_EXTERNAL;
  cfg.frame_delay = FS_MAX_FRAME_DELAY + 1;
  CHECK(fs_create(&cfg, &h) == FS_E_INVALID && !h, "frame_delay above the maximum accepted");
  cfg.frame_delay = 0;
  CHECK(fs_create(&cfg, &h) == FS_OK && h, "fs_create");
  if (!h) return;
  uint8_t p1[8] = {0};
  CHECK(fs_step(h, nullptr, nullptr, FS_ACT_HOST) == FS_E_INVALID, "null p1 accepted");
  CHECK(fs_step(h, p1, nullptr, FS_ACT_HOST) == FS_E_INVALID, "external P2 without actions accepted");
  CHECK(fs_last_error(h) && fs_last_error(h)[0], "no message");
  CHECK(fs_step(h, p1, p1, 5) == FS_E_INVALID, "bad flags accepted");
  CHECK(fs_step_n(h, 0, nullptr, nullptr, 0, nullptr) == FS_E_INVALID, "n = 0 accepted");
  CHECK(fs_step_n_policy(h, 4, nullptr, p1, nullptr) == FS_E_INVALID, "policy without weights accepted");
  CHECK(fs_pack_outputs(h, nullptr) == FS_E_INVALID, "null pack destination accepted");
  fs_destroy(h);
  fs_destroy(nullptr);
}

int main() {
  or_set_threads(4);
  error_paths();
  lockstep(FS_P2_EXTERNAL, FS_AUTORESET_SAME_STEP, FS_FLOAT_STRICT32, 2048, 300, 200);
  lockstep(FS_P2_BOT, FS_AUTORESET_NEXT_STEP, FS_FLOAT_STRICT32, 2048, 300, 200);
  lockstep(FS_P2_NOOP, FS_AUTORESET_SAME_STEP, FS_FLOAT_DOUBLE, 1000, 200, 0);
  determinism_and_pack(3000);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    fflush(stderr);
    return 1;
  }
  printf("abi_lockstep: all checks passed\n");
  fflush(stdout);
  return 0;
}
