// fs_api.cpp -- host side of libfootsies.so: the extern "C" entry points of
// include/footsies.h over the HIP kernels in fs_kernels.hip.
//
// One handle owns one device, one non-blocking HIP stream, the arena state in
// HBM and the output buffers.  Nothing here touches the simulation semantics;
// see fs_kernels.hip.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <link.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "fs_internal.h"

#define FS_API extern "C" __attribute__((visibility("default")))

namespace {

thread_local std::string g_create_error;

struct Buffers {
  // outputs (library-owned)
  uint8_t *guard = nullptr, *move = nullptr, *action = nullptr, *hitstun = nullptr, *terminated = nullptr,
          *truncated = nullptr;
  float *move_frame = nullptr, *position = nullptr;
  double* reward = nullptr;
  int32_t* frame = nullptr;
  uint8_t *f_guard = nullptr, *f_move = nullptr, *f_action = nullptr, *f_hitstun = nullptr;
  float *f_move_frame = nullptr, *f_position = nullptr;
  int32_t* f_frame = nullptr;
};

}  // namespace

struct fs_context {
  fs_config cfg{};
  int n = 0;
  int device = 0;
  hipStream_t stream = nullptr;      // the stream all work is issued on
  hipStream_t own_stream = nullptr;  // the library's own stream
  fsk::DevState st{};
  Buffers own{};
  fsk::DevOutputs out{};  // what the kernels write (own buffers or caller-bound ones)
  // staging for host-side actions / reset arguments
  uint8_t* d_act = nullptr;      // [2][N]
  uint8_t* h_act = nullptr;      // pinned [2][N]
  uint64_t* d_seeds = nullptr;   // [N]
  uint64_t* h_seeds = nullptr;   // pinned [N]
  uint8_t* d_mask = nullptr;     // [N]
  uint8_t* h_mask = nullptr;     // pinned [N]
  hipEvent_t staging_free = nullptr;
  uint4* delay_ring = nullptr;   // frame_delay > 0: [d][N] x 32-B observation records (fs_delay.hip)
  uint8_t* delay_head = nullptr; // frame_delay > 0: [N] each arena's ring head
  std::vector<uint8_t> p2bot;    // host mirror of each arena's P2 actor (1 = the bot)
  bool geom = false;             // the last fs_set_state loaded a fighter with position.y != 0 or a flipped
                                 // facing: steps run the kernels' general-geometry tick
  int p2bot_count = 0;
  std::vector<void*> allocations;
  uint64_t steps = 0;
  std::string err;
};

namespace {

int set_err(fs_context* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  else g_create_error = buf;
  return code;
}

#define HIP_TRY(h, expr)                                                                              \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) return set_err((h), FS_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <typename T>
int dalloc(fs_context* h, T** p, size_t count) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, count * sizeof(T) ? count * sizeof(T) : 1);
  if (e != hipSuccess) return set_err(h, FS_E_OOM, "hipMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
  h->allocations.push_back(q);
  *p = static_cast<T*>(q);
  return FS_OK;
}

void free_all(fs_context* h) {
  for (void* p : h->allocations) (void)hipFree(p);
  h->allocations.clear();
  if (h->h_act) (void)hipHostFree(h->h_act);
  if (h->h_seeds) (void)hipHostFree(h->h_seeds);
  if (h->h_mask) (void)hipHostFree(h->h_mask);
  if (h->staging_free) (void)hipEventDestroy(h->staging_free);
  if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
  h->own_stream = nullptr;
  h->h_act = nullptr;
  h->h_seeds = nullptr;
  h->h_mask = nullptr;
  h->staging_free = nullptr;
  h->stream = nullptr;
}

// The kernel variant for the handle's actors (fs_internal.h): the uniform ones unless P1 is the
// bot or some arena's P2 was switched to the bot.
int variant(const fs_context* h) {
  if (h->cfg.p1_mode == FS_P1_BOT || (h->cfg.p2_mode == FS_P2_EXTERNAL && h->p2bot_count > 0)) return fsk::kActors;
  return h->cfg.p2_mode;
}

void set_p2bot_mirror(fs_context* h, size_t i, uint8_t bot) {
  h->p2bot_count += (int)(bot != 0) - (int)(h->p2bot[i] != 0);
  h->p2bot[i] = bot != 0;
}

int use_device(fs_context* h) {
  int cur = -1;  // (the calling thread is usually on the handle's device already: no hipSetDevice)
  if (hipGetDevice(&cur) == hipSuccess && cur == h->device) return FS_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  return FS_OK;
}

void outputs_from_own(fs_context* h) {
  Buffers& b = h->own;
  h->out = fsk::DevOutputs{b.guard,   b.move,   b.move_frame, b.position,     b.reward,     b.terminated,
                           b.truncated, b.frame, b.action,    b.hitstun,      b.f_guard,    b.f_move,
                           b.f_move_frame, b.f_position, b.f_frame, b.f_action, b.f_hitstun};
}

// FootsiesEnv's delayed-frame queue over rows the last kernel wrote (no-op for frame_delay 0)
int apply_delay(fs_context* h, const fsk::DevOutputs& out, int n_steps, int stride, bool refill_only,
                const uint8_t* active = nullptr) {
  if (h->cfg.frame_delay <= 0) return FS_OK;
  fsk::DelayParams dp{};
  dp.out = out;
  dp.ring = h->delay_ring;
  dp.n_envs = h->n;
  dp.delay = h->cfg.frame_delay;
  dp.n_steps = n_steps;
  dp.out_stride_steps = stride;
  dp.head = h->delay_head;
  dp.active = active;
  dp.refill_only = refill_only ? 1 : 0;
  dp.same_step = h->cfg.autoreset_mode == FS_AUTORESET_SAME_STEP;
  HIP_TRY(h, fsk::launch_delay(dp, h->stream));
  return FS_OK;
}

// wait until the pinned staging buffers may be overwritten
int staging_wait(fs_context* h) {
  HIP_TRY(h, hipEventSynchronize(h->staging_free));
  return FS_OK;
}

// The HIP / HSA runtime images mapped into this process (dl_iterate_phdr), "hip:" / "hsa:" + path
// per line.  Two images of one runtime (e.g. /opt/rocm's libamdhip64 beside the copy bundled with
// a torch wheel, mapped by an extension loaded before torch) each see their own device list, and
// the one this library bound to reports no device (profiles/r05q_lib_before_torch.log).
struct RuntimeImages {
  std::vector<std::string> hip, hsa;
};

int collect_image(struct dl_phdr_info* info, size_t, void* arg) {
  auto* r = static_cast<RuntimeImages*>(arg);
  const char* path = info->dlpi_name;
  if (!path || !*path) return 0;
  const char* base = strrchr(path, '/');
  base = base ? base + 1 : path;
  auto add = [&](std::vector<std::string>& v) {
    char real[4096];
    std::string p = realpath(path, real) ? std::string(real) : std::string(path);
    if (std::find(v.begin(), v.end(), p) == v.end()) v.push_back(p);
  };
  if (!strncmp(base, "libamdhip64.so", 14)) add(r->hip);
  else if (!strncmp(base, "libhsa-runtime64.so", 19)) add(r->hsa);
  return 0;
}

RuntimeImages runtime_images() {
  RuntimeImages r;
  dl_iterate_phdr(collect_image, &r);
  return r;
}

}  // namespace

FS_API int fs_abi_version(void) { return FS_ABI_VERSION; }

FS_API int fs_runtime_images(char* buf, size_t len) {
  RuntimeImages r = runtime_images();
  std::string s;
  for (auto& p : r.hip) s += "hip:" + p + "\n";
  for (auto& p : r.hsa) s += "hsa:" + p + "\n";
  if (buf && len) {
    size_t n = std::min(len - 1, s.size());
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int)std::max(r.hip.size(), r.hsa.size());
}

FS_API int fs_runtime_version(int* runtime, int* build) {
  if (build) *build = HIP_VERSION;
  int v = 0;
  hipError_t e = hipRuntimeGetVersion(&v);
  if (runtime) *runtime = e == hipSuccess ? v : 0;
  return e == hipSuccess ? FS_OK : set_err(nullptr, FS_E_DEVICE, "hipRuntimeGetVersion: %s", hipGetErrorString(e));
}

FS_API int fs_create(const fs_config* cfg, fs_handle* out) {
  g_create_error.clear();
  if (!cfg || !out) return set_err(nullptr, FS_E_INVALID, "fs_create: null argument");
  *out = nullptr;
  if (cfg->num_envs <= 0) return set_err(nullptr, FS_E_INVALID, "num_envs must be > 0 (got %d)", cfg->num_envs);
  if (cfg->p2_mode < FS_P2_EXTERNAL || cfg->p2_mode > FS_P2_NOOP)
    return set_err(nullptr, FS_E_INVALID, "invalid p2_mode %d", cfg->p2_mode);
  if (cfg->p1_mode != FS_P1_EXTERNAL && cfg->p1_mode != FS_P1_BOT)
    return set_err(nullptr, FS_E_INVALID, "invalid p1_mode %d", cfg->p1_mode);
  if (cfg->float_mode != FS_FLOAT_STRICT32 && cfg->float_mode != FS_FLOAT_DOUBLE)
    return set_err(nullptr, FS_E_INVALID, "invalid float_mode %d", cfg->float_mode);
  if (cfg->autoreset_mode != FS_AUTORESET_SAME_STEP && cfg->autoreset_mode != FS_AUTORESET_NEXT_STEP)
    return set_err(nullptr, FS_E_INVALID, "invalid autoreset_mode %d", cfg->autoreset_mode);
  if (cfg->frame_delay < 0 || cfg->frame_delay > FS_MAX_FRAME_DELAY)
    return set_err(nullptr, FS_E_INVALID, "frame_delay must be in [0, %d] (got %d)", FS_MAX_FRAME_DELAY,
                   cfg->frame_delay);
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) {
    RuntimeImages r = runtime_images();
    if (r.hip.size() > 1 || r.hsa.size() > 1) {
      const std::vector<std::string>& v = r.hip.size() > 1 ? r.hip : r.hsa;
      return set_err(nullptr, FS_E_RUNTIME,
                     "two %s runtimes are loaded in this process (%s and %s): the one libfootsies bound to sees no "
                     "device.  Load the HIP runtime the rest of the process uses first (import torch before "
                     "libfootsies), or run with one ROCm installation",
                     r.hip.size() > 1 ? "HIP" : "HSA", v[0].c_str(), v[1].c_str());
    }
    return set_err(nullptr, FS_E_DEVICE, "no HIP device available (%s)", hipGetErrorString(e));
  }
  if (cfg->device_id < 0 || cfg->device_id >= ndev)
    return set_err(nullptr, FS_E_INVALID, "device_id %d out of range (%d devices)", cfg->device_id, ndev);

  fs_context* h = new (std::nothrow) fs_context();
  if (!h) return set_err(nullptr, FS_E_OOM, "out of host memory");
  h->cfg = *cfg;
  h->n = cfg->num_envs;
  h->device = cfg->device_id;
  const size_t N = (size_t)h->n;
  int rc = FS_OK;
  auto fail = [&](int code) {
    std::string msg = h->err;
    free_all(h);
    delete h;
    g_create_error = msg;
    return code;
  };
  if ((rc = use_device(h)) != FS_OK) return fail(rc);
  if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(h, FS_E_DEVICE, "hipStreamCreate failed"));
  h->stream = h->own_stream;
  if (hipEventCreateWithFlags(&h->staging_free, hipEventDisableTiming) != hipSuccess)
    return fail(set_err(h, FS_E_DEVICE, "hipEventCreate failed"));
  // state
  if ((rc = dalloc(h, &h->st.pos, N)) || (rc = dalloc(h, &h->st.hist, N)) || (rc = dalloc(h, &h->st.fpk, N)) ||
      (rc = dalloc(h, &h->st.aw, N)) || (rc = dalloc(h, &h->st.cum, N)))
    return fail(rc);
  // the game RNG and both BattleAIs exist in every mode (a P2 bot can be switched in later)
  if ((rc = dalloc(h, &h->st.rng, N)) || (rc = dalloc(h, &h->st.bot, N)) || (rc = dalloc(h, &h->st.bot1, N)) ||
      (rc = dalloc(h, &h->st.posy, N)))
    return fail(rc);
  h->p2bot.assign(N, cfg->p2_mode == FS_P2_BOT ? 1 : 0);
  h->p2bot_count = cfg->p2_mode == FS_P2_BOT ? h->n : 0;
  // outputs
  Buffers& b = h->own;
  if ((rc = dalloc(h, &b.guard, 2 * N)) || (rc = dalloc(h, &b.move, 2 * N)) || (rc = dalloc(h, &b.action, 2 * N)) ||
      (rc = dalloc(h, &b.hitstun, 2 * N)) || (rc = dalloc(h, &b.terminated, N)) || (rc = dalloc(h, &b.truncated, N)) ||
      (rc = dalloc(h, &b.move_frame, 2 * N)) || (rc = dalloc(h, &b.position, 2 * N)) ||
      (rc = dalloc(h, &b.reward, N)) || (rc = dalloc(h, &b.frame, N)) || (rc = dalloc(h, &b.f_guard, 2 * N)) ||
      (rc = dalloc(h, &b.f_move, 2 * N)) || (rc = dalloc(h, &b.f_action, 2 * N)) ||
      (rc = dalloc(h, &b.f_hitstun, 2 * N)) || (rc = dalloc(h, &b.f_move_frame, 2 * N)) ||
      (rc = dalloc(h, &b.f_position, 2 * N)) || (rc = dalloc(h, &b.f_frame, N)))
    return fail(rc);
  // staging
  if ((rc = dalloc(h, &h->d_act, 2 * N)) || (rc = dalloc(h, &h->d_seeds, N)) || (rc = dalloc(h, &h->d_mask, N)))
    return fail(rc);
  if (cfg->frame_delay > 0 && ((rc = dalloc(h, &h->delay_ring, 2 * (size_t)cfg->frame_delay * N)) ||
                               (rc = dalloc(h, &h->delay_head, N))))
    return fail(rc);
  if (cfg->frame_delay > 0 && hipMemsetAsync(h->delay_head, 0, N, h->stream) != hipSuccess)
    return fail(set_err(h, FS_E_DEVICE, "memset"));
  if (hipHostMalloc((void**)&h->h_act, 2 * N, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h->h_seeds, N * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h->h_mask, N, hipHostMallocDefault) != hipSuccess)
    return fail(set_err(h, FS_E_OOM, "hipHostMalloc failed"));
  outputs_from_own(h);
  // zero the final_* rows so untouched rows read deterministically
  for (void* p : {(void*)b.f_guard, (void*)b.f_move, (void*)b.f_action, (void*)b.f_hitstun})
    if (hipMemsetAsync(p, 0, 2 * N, h->stream) != hipSuccess) return fail(set_err(h, FS_E_DEVICE, "memset"));
  if (hipMemsetAsync(b.f_move_frame, 0, 2 * N * sizeof(float), h->stream) != hipSuccess ||
      hipMemsetAsync(b.f_position, 0, 2 * N * sizeof(float), h->stream) != hipSuccess ||
      hipMemsetAsync(b.f_frame, 0, N * sizeof(int32_t), h->stream) != hipSuccess)
    return fail(set_err(h, FS_E_DEVICE, "memset"));
  if (hipEventRecord(h->staging_free, h->stream) != hipSuccess) return fail(set_err(h, FS_E_DEVICE, "event"));
  // game start: Stop -> Intro -> Fight (state(-1))
  fsk::ResetParams rp{};
  rp.st = h->st;
  rp.out = h->out;
  rp.n_envs = h->n;
  rp.flags = FS_RESET_HARD;
  rp.init = 1;
  rp.base_seed = cfg->base_seed;
  rp.arena_base = cfg->arena_base;
  rp.p1_bot = cfg->p1_mode == FS_P1_BOT;
  rp.p2_mode = cfg->p2_mode;
  hipError_t le = fsk::launch_reset(rp, cfg->float_mode, h->stream);
  if (le != hipSuccess) return fail(set_err(h, FS_E_DEVICE, "reset kernel launch: %s", hipGetErrorString(le)));
  if ((rc = apply_delay(h, h->out, 1, 0, true))) return fail(rc);  // the first reset's queue (FE:502-504)
  le = hipStreamSynchronize(h->stream);
  if (le != hipSuccess) return fail(set_err(h, FS_E_DEVICE, "reset kernel: %s", hipGetErrorString(le)));
  *out = h;
  return FS_OK;
}

FS_API int fs_reset(fs_handle h, const uint64_t* seeds, const uint8_t* mask, int flags) {
  if (!h) return FS_E_INVALID;
  if (flags != FS_RESET_HARD && flags != FS_RESET_IF_NEEDED && flags != FS_RESET_SEED_ONLY)
    return set_err(h, FS_E_INVALID, "bad flags %d", flags);
  if (flags == FS_RESET_SEED_ONLY && !seeds) return FS_OK;
  int rc;
  if ((rc = use_device(h))) return rc;
  if ((rc = staging_wait(h))) return rc;
  const size_t N = (size_t)h->n;
  fsk::ResetParams rp{};
  rp.st = h->st;
  rp.out = h->out;
  rp.n_envs = h->n;
  rp.flags = flags;
  rp.init = 0;
  rp.arena_base = h->cfg.arena_base;
  rp.p1_bot = h->cfg.p1_mode == FS_P1_BOT;
  rp.p2_mode = h->cfg.p2_mode;
  if (seeds) {
    memcpy(h->h_seeds, seeds, N * sizeof(uint64_t));
    HIP_TRY(h, hipMemcpyAsync(h->d_seeds, h->h_seeds, N * sizeof(uint64_t), hipMemcpyHostToDevice, h->stream));
    rp.seeds = h->d_seeds;
  }
  if (mask) {
    memcpy(h->h_mask, mask, N);
    HIP_TRY(h, hipMemcpyAsync(h->d_mask, h->h_mask, N, hipMemcpyHostToDevice, h->stream));
    rp.mask = h->d_mask;
  }
  HIP_TRY(h, hipEventRecord(h->staging_free, h->stream));
  HIP_TRY(h, fsk::launch_reset(rp, h->cfg.float_mode, h->stream));
  if (flags != FS_RESET_SEED_ONLY && (rc = apply_delay(h, h->out, 1, 0, true))) return rc;
  return FS_OK;
}

static int step_common(fs_handle h, int n, const uint8_t* p1, const uint8_t* p2, int flags, uint64_t seed,
                       const fs_outputs* traj, const uint8_t* active = nullptr,
                       const fs_policy* pol = nullptr, const fs_packed_traj* pk = nullptr, void* rec = nullptr) {
  int rc;
  if ((rc = use_device(h))) return rc;
  const size_t N = (size_t)h->n;
  fsk::StepParams sp{};
  sp.st = h->st;
  sp.out = h->out;
  sp.n_envs = h->n;
  sp.n_steps = n;
  sp.out_stride_steps = 0;
  sp.dense_reward = h->cfg.dense_reward;
  sp.autoreset_mode = h->cfg.autoreset_mode;
  sp.action_seed = seed;
  sp.t0 = h->steps;
  sp.arena_base = h->cfg.arena_base;
  sp.p1_bot = h->cfg.p1_mode == FS_P1_BOT;
  sp.p2_resets = h->cfg.p2_mode == FS_P2_BOT;
  sp.p2_noop = h->cfg.p2_mode == FS_P2_NOOP;
  sp.geom = h->geom;
  sp.rec = static_cast<uint2*>(rec);  // (one-tick launches only: fs_step_rec)
  if (pol) sp.pol = fsk::PolicyParams{pol->w1, pol->b1, pol->w2, pol->b2, pol->w3, pol->b3,
                                      pol->actions_out, pol->logp_out, pol->seed};
  const bool ext = h->cfg.p2_mode == FS_P2_EXTERNAL;
  const bool p1_bot = h->cfg.p1_mode == FS_P1_BOT;
  if (flags == FS_ACT_HOST && (p1 || p1_bot) && !active && N <= (size_t)fsk::kInlineArenas) {
    // a few arenas (the single-env drop-in): the inputs travel in the kernel arguments, so the
    // launch does not wait behind a host-to-device copy (one-arena step 20.7 -> 13.5 us when it
    // is the only copy, tools/single_env_probe.py)
    if (n != 1) return set_err(h, FS_E_INVALID, "host actions are only accepted for single steps");
    sp.inl_n = (int)N;
    if (p1) memcpy(sp.inl[0], p1, N);
    if (ext) memcpy(sp.inl[1], p2, N);
    sp.p1 = h->d_act;  // (not read: non-null so that the row kernels, not the hashed one, run)
    sp.p2 = ext ? h->d_act + N : nullptr;
    sp.active = nullptr;
  } else if (flags == FS_ACT_HOST && (p1 || p1_bot)) {
    if (n != 1) return set_err(h, FS_E_INVALID, "host actions are only accepted for single steps");
    if ((rc = staging_wait(h))) return rc;
    if (p1) memcpy(h->h_act, p1, N);
    else memset(h->h_act, 0, N);  // P1 is the bot: the row is not read
    if (ext) memcpy(h->h_act + N, p2, N);
    HIP_TRY(h, hipMemcpyAsync(h->d_act, h->h_act, ext ? 2 * N : N, hipMemcpyHostToDevice, h->stream));
    if (active) {
      memcpy(h->h_mask, active, N);
      HIP_TRY(h, hipMemcpyAsync(h->d_mask, h->h_mask, N, hipMemcpyHostToDevice, h->stream));
    }
    HIP_TRY(h, hipEventRecord(h->staging_free, h->stream));
    sp.p1 = h->d_act;
    sp.p2 = ext ? h->d_act + N : nullptr;
    sp.active = active ? h->d_mask : nullptr;
  } else {
    // P1 bot with explicit P2 rows (or records to write, which only k_step does): P1's row is
    // never read, but a null p1 would select the hashed-action kernel, so it points at the staging row
    sp.p1 = (p1_bot && !p1 && (p2 || rec)) ? h->d_act : p1;
    sp.p2 = ext ? p2 : nullptr;
    sp.active = active;
  }
  if (traj) {
    sp.out = fsk::DevOutputs{traj->guard,          traj->move,           traj->move_frame,  traj->position,
                             traj->reward,         traj->terminated,     traj->truncated,   traj->frame,
                             traj->action,         traj->hitstun,        traj->final_guard, traj->final_move,
                             traj->final_move_frame, traj->final_position, traj->final_frame, traj->final_action,
                             traj->final_hitstun};
    const void* req[] = {traj->guard, traj->move,   traj->move_frame, traj->position, traj->reward,
                         traj->terminated, traj->truncated, traj->frame, traj->action, traj->hitstun};
    for (const void* q : req)
      if (!q) return set_err(h, FS_E_INVALID, "fs_step_n: trajectory buffer missing");
    if (h->cfg.autoreset_mode == FS_AUTORESET_SAME_STEP &&
        (!traj->final_guard || !traj->final_move || !traj->final_move_frame || !traj->final_position ||
         !traj->final_frame || !traj->final_action || !traj->final_hitstun))
      return set_err(h, FS_E_INVALID, "fs_step_n: final_* trajectory buffers required in same-step autoreset");
    sp.out_stride_steps = 1;
  } else if (pk) {  // (fs_step_n_packed validated the buffers)
    sp.out = fsk::DevOutputs{};
    sp.out.reward = pk->reward;
    sp.out.pk_lanes = static_cast<uint4*>(pk->lanes);
    sp.out.pk_final = static_cast<uint4*>(pk->final_lanes);
    sp.out_stride_steps = 1;
  } else if (n > 1 && h->cfg.frame_delay > 0) {
    // the delayed queue needs every step's row, which a fused launch without a
    // trajectory overwrites: step one tick per launch instead
    for (int j = 0; j < n; j++) {
      const uint8_t* q1 = sp.p1 ? sp.p1 + (size_t)j * N : nullptr;
      const uint8_t* q2 = sp.p2 ? sp.p2 + (size_t)j * N : nullptr;
      if ((rc = step_common(h, 1, q1 ? q1 : (p1_bot ? h->d_act : nullptr), q2, FS_ACT_DEVICE, seed, nullptr)))
        return rc;
    }
    return FS_OK;
  }
  HIP_TRY(h, fsk::launch_step(sp, h->cfg.float_mode, variant(h), h->stream));
  if ((rc = apply_delay(h, sp.out, n, sp.out_stride_steps, false, sp.active))) return rc;
  h->steps += (uint64_t)n;
  return FS_OK;
}

// The kernels address trajectory rows with 32-bit byte offsets (row t of arena a at
// (t * N + a) * element size, up to 8 B for the f64 reward), so one launch covers at most
// kMaxLaunchRows arena-ticks; longer fused calls run as consecutive launches over row ranges
// of the same buffers.  Hashed actions and the actor's sampling stream are keyed by the
// handle's step counter, which each launch advances, so the split is invisible in the results.
constexpr uint64_t kMaxLaunchRows = 0xFFFFFFFFull / 8u;
// (a packed trajectory's lane records: 32 B per row)
constexpr uint64_t kMaxPackedLaunchRows = 0xFFFFFFFFull / 32u;

static int step_chunked(fs_handle h, int n, const uint8_t* p1, const uint8_t* p2, uint64_t seed,
                        const fs_outputs* traj, const fs_policy* pol, const fs_packed_traj* pk = nullptr) {
  const uint64_t N = (uint64_t)h->n;
  uint64_t rows = pk ? kMaxPackedLaunchRows : kMaxLaunchRows;
  if (const char* e = getenv("FOOTSIES_MAX_LAUNCH_ROWS"))  // test hook: exercise the split at small sizes
    rows = std::min<uint64_t>(rows, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
  const int max_n = (int)std::max<uint64_t>(1, std::min<uint64_t>(rows / N, 0x7fffffff));
  if (n <= max_n) return step_common(h, n, p1, p2, FS_ACT_DEVICE, seed, traj, nullptr, pol, pk);
  for (int j = 0; j < n;) {
    const int m = std::min(max_n, n - j);
    const uint64_t row = (uint64_t)j * N;  // first arena-tick row of this launch
    fs_outputs t{};
    if (traj) {
      t = *traj;
      auto adv = [&](auto*& q, uint64_t per_row) { if (q) q += row * per_row; };
      adv(t.guard, 2); adv(t.move, 2); adv(t.move_frame, 2); adv(t.position, 2); adv(t.reward, 1);
      adv(t.terminated, 1); adv(t.truncated, 1); adv(t.frame, 1); adv(t.action, 2); adv(t.hitstun, 2);
      adv(t.final_guard, 2); adv(t.final_move, 2); adv(t.final_move_frame, 2); adv(t.final_position, 2);
      adv(t.final_frame, 1); adv(t.final_action, 2); adv(t.final_hitstun, 2);
    }
    fs_policy q{};
    if (pol) {
      q = *pol;
      if (q.actions_out) q.actions_out += row;
      if (q.logp_out) q.logp_out += row;
    }
    fs_packed_traj k{};
    if (pk) {
      k = *pk;
      k.lanes = static_cast<char*>(k.lanes) + row * 2 * FS_PACKED_LANE_BYTES;
      k.reward += row;
      if (k.final_lanes) k.final_lanes = static_cast<char*>(k.final_lanes) + row * 2 * FS_PACKED_LANE_BYTES;
    }
    const int rc = step_common(h, m, p1 ? p1 + row : nullptr, p2 ? p2 + row : nullptr, FS_ACT_DEVICE, seed,
                               traj ? &t : nullptr, nullptr, pol ? &q : nullptr, pk ? &k : nullptr);
    if (rc) return rc;
    j += m;
  }
  return FS_OK;
}

FS_API int fs_set_p2_mode(fs_handle h, int mode, const uint8_t* mask) {
  if (!h) return FS_E_INVALID;
  if (mode != FS_P2_EXTERNAL && mode != FS_P2_BOT)
    return set_err(h, FS_E_INVALID, "fs_set_p2_mode: mode must be FS_P2_EXTERNAL or FS_P2_BOT (got %d)", mode);
  if (h->cfg.p2_mode != FS_P2_EXTERNAL)
    return set_err(h, FS_E_UNSUPPORTED, "fs_set_p2_mode: the handle needs a remote P2 (FS_P2_EXTERNAL) to switch "
                                        "its opponent (FE:468-470)");
  int rc;
  if ((rc = use_device(h))) return rc;
  const size_t N = (size_t)h->n;
  const uint8_t* dmask = nullptr;
  if (mask) {
    if ((rc = staging_wait(h))) return rc;
    memcpy(h->h_mask, mask, N);
    HIP_TRY(h, hipMemcpyAsync(h->d_mask, h->h_mask, N, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(h, hipEventRecord(h->staging_free, h->stream));
    dmask = h->d_mask;
  }
  HIP_TRY(h, fsk::launch_set_p2(h->st, mode == FS_P2_BOT, dmask, h->n, h->stream));
  for (size_t i = 0; i < N; i++)
    if (!mask || mask[i]) set_p2bot_mirror(h, i, mode == FS_P2_BOT);
  return FS_OK;
}

FS_API int fs_step(fs_handle h, const uint8_t* p1_act, const uint8_t* p2_act, int flags) {
  if (!h) return FS_E_INVALID;
  if (!p1_act && h->cfg.p1_mode != FS_P1_BOT) return set_err(h, FS_E_INVALID, "fs_step: p1 actions required");
  if (h->cfg.p2_mode == FS_P2_EXTERNAL && !p2_act)
    return set_err(h, FS_E_INVALID, "fs_step: p2 actions required for FS_P2_EXTERNAL");
  if (flags != FS_ACT_HOST && flags != FS_ACT_DEVICE) return set_err(h, FS_E_INVALID, "bad flags %d", flags);
  return step_common(h, 1, p1_act, p2_act, flags, 0, nullptr);
}

FS_API int fs_step_rec(fs_handle h, const uint8_t* p1_act, const uint8_t* p2_act, int flags, void* rec) {
  if (!h) return FS_E_INVALID;
  if (!rec) return set_err(h, FS_E_INVALID, "fs_step_rec: record destination required");
  if (reinterpret_cast<uintptr_t>(rec) % 8) return set_err(h, FS_E_INVALID, "fs_step_rec: records must be 8-byte aligned");
  if (h->cfg.frame_delay > 0) {  // (the delayed queue rewrites the outputs after the tick: pack those)
    const int rc = fs_step(h, p1_act, p2_act, flags);
    return rc ? rc : fs_pack_outputs(h, rec);
  }
  if (!p1_act && h->cfg.p1_mode != FS_P1_BOT) return set_err(h, FS_E_INVALID, "fs_step_rec: p1 actions required");
  if (h->cfg.p2_mode == FS_P2_EXTERNAL && !p2_act)
    return set_err(h, FS_E_INVALID, "fs_step_rec: p2 actions required for FS_P2_EXTERNAL");
  if (flags != FS_ACT_HOST && flags != FS_ACT_DEVICE) return set_err(h, FS_E_INVALID, "bad flags %d", flags);
  return step_common(h, 1, p1_act, p2_act, flags, 0, nullptr, nullptr, nullptr, nullptr, rec);
}

FS_API int fs_step_masked(fs_handle h, const uint8_t* p1_act, const uint8_t* p2_act, const uint8_t* active,
                          int flags) {
  if (!h) return FS_E_INVALID;
  if ((!p1_act && h->cfg.p1_mode != FS_P1_BOT) || !active)
    return set_err(h, FS_E_INVALID, "fs_step_masked: p1 actions and mask required");
  if (h->cfg.p2_mode == FS_P2_EXTERNAL && !p2_act)
    return set_err(h, FS_E_INVALID, "fs_step_masked: p2 actions required for FS_P2_EXTERNAL");
  if (flags != FS_ACT_HOST && flags != FS_ACT_DEVICE) return set_err(h, FS_E_INVALID, "bad flags %d", flags);
  return step_common(h, 1, p1_act, p2_act, flags, 0, nullptr, active);
}

FS_API int fs_step_n(fs_handle h, int n, const uint8_t* p1_act, const uint8_t* p2_act, uint64_t action_seed,
                     const fs_outputs* traj) {
  if (!h) return FS_E_INVALID;
  if (n <= 0) return set_err(h, FS_E_INVALID, "fs_step_n: n must be > 0");
  if ((p1_act == nullptr) != (p2_act == nullptr) && h->cfg.p2_mode == FS_P2_EXTERNAL &&
      !(p1_act == nullptr && h->cfg.p1_mode == FS_P1_BOT))
    return set_err(h, FS_E_INVALID, "fs_step_n: give both action arrays or neither");
  return step_chunked(h, n, p1_act, p2_act, action_seed, traj, nullptr);
}

FS_API int fs_step_n_packed(fs_handle h, int n, const uint8_t* p1_act, const uint8_t* p2_act,
                            const fs_packed_traj* traj) {
  if (!h) return FS_E_INVALID;
  if (n <= 0) return set_err(h, FS_E_INVALID, "fs_step_n_packed: n must be > 0");
  if (!p1_act) return set_err(h, FS_E_INVALID, "fs_step_n_packed: p1 action rows required");
  if (h->cfg.p2_mode == FS_P2_EXTERNAL && !p2_act)
    return set_err(h, FS_E_INVALID, "fs_step_n_packed: p2 action rows required for FS_P2_EXTERNAL");
  if (!traj || !traj->lanes || !traj->reward)
    return set_err(h, FS_E_INVALID, "fs_step_n_packed: lanes and reward buffers required");
  if (h->cfg.autoreset_mode == FS_AUTORESET_SAME_STEP && !traj->final_lanes)
    return set_err(h, FS_E_INVALID, "fs_step_n_packed: final_lanes required in same-step autoreset");
  if (reinterpret_cast<uintptr_t>(traj->lanes) % 16 || reinterpret_cast<uintptr_t>(traj->final_lanes) % 16 ||
      reinterpret_cast<uintptr_t>(traj->reward) % 8)
    return set_err(h, FS_E_INVALID, "fs_step_n_packed: lanes / final_lanes must be 16-byte, reward 8-byte aligned");
  if (h->cfg.frame_delay > 0)
    return set_err(h, FS_E_UNSUPPORTED, "fs_step_n_packed: frame_delay > 0 is not supported (the delayed queue "
                                        "reads the per-field outputs)");
  return step_chunked(h, n, p1_act, p2_act, 0, nullptr, nullptr, traj);
}

FS_API int fs_step_n_policy(fs_handle h, int n, const fs_policy* pol, const uint8_t* p2_act,
                            const fs_outputs* traj) {
  if (!h) return FS_E_INVALID;
  if (!pol || !pol->w1 || !pol->b1 || !pol->w2 || !pol->b2 || !pol->w3 || !pol->b3)
    return set_err(h, FS_E_INVALID, "fs_step_n_policy: all six weight arrays required");
  if (n <= 0) return set_err(h, FS_E_INVALID, "fs_step_n_policy: n must be > 0");
  if (h->cfg.p1_mode == FS_P1_BOT)
    return set_err(h, FS_E_UNSUPPORTED, "fs_step_n_policy: P1 is the bot (FS_P1_BOT), not the actor");
  if (h->cfg.p2_mode == FS_P2_EXTERNAL && !p2_act)
    return set_err(h, FS_E_INVALID, "fs_step_n_policy: p2 actions required for FS_P2_EXTERNAL");
  if (h->cfg.frame_delay > 0)
    return set_err(h, FS_E_UNSUPPORTED, "fs_step_n_policy: the actor observes undelayed frames; frame_delay > 0 "
                                        "is not supported");
  return step_chunked(h, n, nullptr, p2_act, 0, traj, pol);
}

FS_API size_t fs_ppo_workspace_bytes(void) { return fsk::ppo_workspace_bytes(); }

static int ppo_grad(const float* rows, int64_t n, const fs_mlp* actor, const fs_mlp* critic, float clip,
                    float vf_coef, float ent_coef, float* grad_out, float* loss_out, void* workspace,
                    size_t workspace_bytes, void* stream, int precision, const int64_t* runs = nullptr,
                    int run_shift = 0, int64_t n_rows = 0) {
  if (!rows || n <= 0 || !actor || !critic || !grad_out || !loss_out || !workspace)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad: rows, n > 0, both networks, outputs and workspace required");
  if (workspace_bytes < fsk::ppo_workspace_bytes())
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad: workspace of %zu bytes, %zu needed", workspace_bytes,
                   fsk::ppo_workspace_bytes());
  if (precision != FS_PPO_FP32 && precision != FS_PPO_SPLIT_BF16)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad: unknown precision %d", precision);
  if (reinterpret_cast<uintptr_t>(rows) % 16)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad: rows must be 16-byte aligned");
  const float* const a[6] = {actor->w1, actor->b1, actor->w2, actor->b2, actor->w3, actor->b3};
  const float* const c[6] = {critic->w1, critic->b1, critic->w2, critic->b2, critic->w3, critic->b3};
  for (int i = 0; i < 6; ++i)
    if (!a[i] || !c[i]) return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad: all six arrays of each network required");
  const hipError_t e = fsk::launch_ppo_grad(rows, n, a, c, clip, vf_coef, ent_coef, grad_out, loss_out, workspace,
                                            static_cast<hipStream_t>(stream), precision == FS_PPO_SPLIT_BF16, runs,
                                            run_shift, n_rows);
  if (e != hipSuccess) return set_err(nullptr, FS_E_DEVICE, "fs_ppo_grad: %s", hipGetErrorString(e));
  return FS_OK;
}

FS_API int fs_ppo_grad_ex(const float* rows, int64_t n, const fs_mlp* actor, const fs_mlp* critic, float clip,
                          float vf_coef, float ent_coef, float* grad_out, float* loss_out, void* workspace,
                          size_t workspace_bytes, void* stream, int precision) {
  return ppo_grad(rows, n, actor, critic, clip, vf_coef, ent_coef, grad_out, loss_out, workspace, workspace_bytes,
                  stream, precision);
}

FS_API int fs_ppo_grad_runs(const float* rows, int64_t n_rows, const int64_t* runs, int64_t n_runs, int run_shift,
                            const fs_mlp* actor, const fs_mlp* critic, float clip, float vf_coef, float ent_coef,
                            float* grad_out, float* loss_out, void* workspace, size_t workspace_bytes, void* stream,
                            int precision) {
  if (!runs || n_runs <= 0 || n_rows <= 0 || run_shift < 0 || run_shift > 30)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad_runs: runs, n_runs > 0, n_rows > 0 and run_shift in [0, 30] "
                                          "required");
  if (n_runs > (INT64_MAX >> run_shift) || (n_rows >> run_shift) < 1)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_grad_runs: %lld runs of 2^%d rows do not fit a %lld-row table",
                   (long long)n_runs, run_shift, (long long)n_rows);
  return ppo_grad(rows, n_runs << run_shift, actor, critic, clip, vf_coef, ent_coef, grad_out, loss_out, workspace,
                  workspace_bytes, stream, precision, runs, run_shift, n_rows);
}

FS_API int fs_ppo_grad(const float* rows, int64_t n, const fs_mlp* actor, const fs_mlp* critic, float clip,
                       float vf_coef, float ent_coef, float* grad_out, float* loss_out, void* workspace,
                       size_t workspace_bytes, void* stream) {
  return fs_ppo_grad_ex(rows, n, actor, critic, clip, vf_coef, ent_coef, grad_out, loss_out, workspace,
                        workspace_bytes, stream, FS_PPO_FP32);
}

FS_API int fs_ppo_eval_ex(const float* x, int64_t n_values, const uint8_t* actions, int64_t n_logp,
                          const fs_mlp* actor, const fs_mlp* critic, float* values_out, float* logp_out,
                          void* workspace, size_t workspace_bytes, void* stream, int precision) {
  if (!x || n_values <= 0 || n_logp < 0 || n_logp > n_values)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: x, n_values > 0 and 0 <= n_logp <= n_values required");
  if (reinterpret_cast<uintptr_t>(x) % 16) return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: x must be 16-byte aligned");
  if (values_out && !critic) return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: values_out needs the critic");
  if (logp_out && n_logp > 0 && (!actor || !actions))
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: logp_out needs the actor and actions");
  if (precision != FS_PPO_FP32 && precision != FS_PPO_SPLIT_BF16)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: unknown precision %d", precision);
  if (precision == FS_PPO_SPLIT_BF16 && (!workspace || workspace_bytes < fsk::ppo_workspace_bytes()))
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: split-bf16 needs a workspace of %zu bytes",
                   fsk::ppo_workspace_bytes());
  const fs_mlp none{};
  const fs_mlp& A = actor ? *actor : none;
  const fs_mlp& Cn = critic ? *critic : none;
  const float* const a[6] = {A.w1, A.b1, A.w2, A.b2, A.w3, A.b3};
  const float* const c[6] = {Cn.w1, Cn.b1, Cn.w2, Cn.b2, Cn.w3, Cn.b3};
  for (int i = 0; i < 6; ++i)
    if ((values_out && !c[i]) || (logp_out && n_logp > 0 && !a[i]))
      return set_err(nullptr, FS_E_INVALID, "fs_ppo_eval: all six arrays of each network used required");
  const hipError_t e = fsk::launch_ppo_eval(x, n_values, actions, n_logp, a, c, values_out, logp_out, workspace,
                                            static_cast<hipStream_t>(stream), precision == FS_PPO_SPLIT_BF16);
  if (e != hipSuccess) return set_err(nullptr, FS_E_DEVICE, "fs_ppo_eval: %s", hipGetErrorString(e));
  return FS_OK;
}

FS_API int fs_ppo_eval(const float* x, int64_t n_values, const uint8_t* actions, int64_t n_logp, const fs_mlp* actor,
                       const fs_mlp* critic, float* values_out, float* logp_out, void* stream) {
  return fs_ppo_eval_ex(x, n_values, actions, n_logp, actor, critic, values_out, logp_out, nullptr, 0, stream,
                        FS_PPO_FP32);
}

FS_API int fs_ppo_gae(const double* rewards, const uint8_t* done, const float* values, int T, int64_t N, float gamma,
                      float gamma_lam, float* adv_out, float* ret_out, void* stream) {
  if (!rewards || !done || !values || !adv_out || !ret_out || T <= 0 || N <= 0)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_gae: all five arrays, T > 0 and N > 0 required");
  const hipError_t e = fsk::launch_ppo_gae(rewards, done, values, T, N, gamma, gamma_lam, adv_out, ret_out,
                                           static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return set_err(nullptr, FS_E_DEVICE, "fs_ppo_gae: %s", hipGetErrorString(e));
  return FS_OK;
}

FS_API int fs_ppo_features(const uint8_t* guard, const uint8_t* move, const float* move_frame, const float* position,
                           int64_t n, float* out, void* stream) {
  if (!guard || !move || !move_frame || !position || !out || n <= 0)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_features: all five arrays and n > 0 required");
  if (reinterpret_cast<uintptr_t>(out) % 16 || reinterpret_cast<uintptr_t>(move_frame) % 8 ||
      reinterpret_cast<uintptr_t>(position) % 8 || reinterpret_cast<uintptr_t>(guard) % 2 ||
      reinterpret_cast<uintptr_t>(move) % 2)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_features: misaligned array");
  const hipError_t e = fsk::launch_ppo_features(guard, move, move_frame, position, n, out,
                                                static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return set_err(nullptr, FS_E_DEVICE, "fs_ppo_features: %s", hipGetErrorString(e));
  return FS_OK;
}

FS_API int fs_ppo_pack(const float* x, const uint8_t* actions, const float* old_logp, const float* adv,
                       const float* ret, const float* stats, int64_t n, float* rows_out, void* stream) {
  if (!x || !actions || !old_logp || !adv || !ret || !stats || !rows_out || n <= 0)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_pack: all seven arrays and n > 0 required");
  if (reinterpret_cast<uintptr_t>(x) % 16 || reinterpret_cast<uintptr_t>(rows_out) % 16)
    return set_err(nullptr, FS_E_INVALID, "fs_ppo_pack: x and rows_out must be 16-byte aligned");
  const hipError_t e = fsk::launch_ppo_pack(x, actions, old_logp, adv, ret, stats, n, rows_out,
                                            static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return set_err(nullptr, FS_E_DEVICE, "fs_ppo_pack: %s", hipGetErrorString(e));
  return FS_OK;
}

FS_API int fs_hash_actions(fs_handle h, int n_steps, uint64_t seed, uint64_t t0, uint8_t* p1_out, uint8_t* p2_out) {
  if (!h || !p1_out || n_steps <= 0) return FS_E_INVALID;
  int rc;
  if ((rc = use_device(h))) return rc;
  HIP_TRY(h, fsk::launch_hash_actions(h->n, n_steps, seed, t0, h->cfg.arena_base, p1_out, p2_out, h->stream));
  return FS_OK;
}

FS_API int fs_outputs_get(fs_handle h, fs_outputs* o) {
  if (!h || !o) return FS_E_INVALID;
  const fsk::DevOutputs& d = h->out;
  *o = fs_outputs{d.guard,        d.move,           d.move_frame,  d.position,     d.reward,       d.terminated,
                  d.truncated,    d.frame,          d.action,      d.hitstun,      d.final_guard,  d.final_move,
                  d.final_move_frame, d.final_position, d.final_frame, d.final_action, d.final_hitstun};
  return FS_OK;
}

FS_API int fs_pack_outputs(fs_handle h, void* dst) {
  if (!h) return FS_E_INVALID;
  if (!dst) return set_err(h, FS_E_INVALID, "fs_pack_outputs: destination required");
  int rc;
  if ((rc = use_device(h))) return rc;
  HIP_TRY(h, fsk::launch_pack_records(h->out, dst, h->n, h->stream));
  return FS_OK;
}

FS_API int fs_bind_outputs(fs_handle h, const fs_outputs* dev) {
  if (!h) return FS_E_INVALID;
  outputs_from_own(h);
  if (!dev) return FS_OK;
#define BIND(f, g) \
  if (dev->f) h->out.g = dev->f
  BIND(guard, guard);
  BIND(move, move);
  BIND(move_frame, move_frame);
  BIND(position, position);
  BIND(reward, reward);
  BIND(terminated, terminated);
  BIND(truncated, truncated);
  BIND(frame, frame);
  BIND(action, action);
  BIND(hitstun, hitstun);
  BIND(final_guard, final_guard);
  BIND(final_move, final_move);
  BIND(final_move_frame, final_move_frame);
  BIND(final_position, final_position);
  BIND(final_frame, final_frame);
  BIND(final_action, final_action);
  BIND(final_hitstun, final_hitstun);
#undef BIND
  return FS_OK;
}

FS_API int fs_get_env_state(fs_handle h, fs_env_state* host_out) {
  if (!h || !host_out) return FS_E_INVALID;
  int rc;
  if ((rc = use_device(h))) return rc;
  fs_env_state* d = nullptr;
  HIP_TRY(h, hipMalloc(&d, sizeof(fs_env_state) * (size_t)h->n));
  hipError_t e = fsk::launch_get_state(h->st, nullptr, d, h->n, h->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(host_out, d, sizeof(fs_env_state) * (size_t)h->n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return set_err(h, FS_E_DEVICE, "fs_get_env_state: %s", hipGetErrorString(e));
  return FS_OK;
}

FS_API int fs_get_state(fs_handle h, fs_arena_state* host_out) {
  if (!h || !host_out) return FS_E_INVALID;
  int rc;
  if ((rc = use_device(h))) return rc;
  fs_arena_state* d = nullptr;
  HIP_TRY(h, hipMalloc(&d, sizeof(fs_arena_state) * (size_t)h->n));
  hipError_t e = fsk::launch_get_state(h->st, d, nullptr, h->n, h->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(host_out, d, sizeof(fs_arena_state) * (size_t)h->n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return set_err(h, FS_E_DEVICE, "fs_get_state: %s", hipGetErrorString(e));
  return FS_OK;
}

static const int32_t kIds[] = {0, 1, 2, 10, 11, 100, 105, 110, 115, 200, 301, 305, 306, 310, 350, 500, 510};
static bool valid_action_id(int32_t id) {
  for (int32_t k : kIds)
    if (k == id) return true;
  return false;
}
// a BattleAI's canonical fields fit the bot word, and a queue index lies inside its plan (an
// index at the end is an empty queue: plan -1)
static bool valid_bot(int32_t mp, int32_t mi, int32_t ap, int32_t ai, int32_t prev_opp) {
  return mp >= -1 && mp <= 6 && ap >= -1 && ap <= 4 && mi >= 0 && mi <= 127 && ai >= 0 && ai <= 127 &&
         valid_action_id(prev_opp) && (mp < 0 || (uint32_t)mi < fsk::move_plan_len((uint32_t)mp)) &&
         (ap < 0 || (uint32_t)ai < fsk::attack_plan_len((uint32_t)ap));
}

FS_API int fs_set_state(fs_handle h, const fs_arena_state* host_in) {
  if (!h || !host_in) return FS_E_INVALID;
  for (int i = 0; i < h->n; i++) {  // the packed layout's ranges (fs_kernels.hip)
    const fs_arena_state& s = host_in[i];
    for (int k = 0; k < 2; k++) {
      const fs_fighter_state& f = s.f[k];
      if (!valid_action_id(f.action_id) || f.action_frame < 0 || f.action_frame > 511 || f.hitstun < 0 ||
          f.hitstun > 31 || f.vital < 0 || f.vital > 3 || f.guard < 0 || f.guard > 3 || f.hit_count < 0 ||
          f.hit_count > 3 || f.attack_hold < 0 || f.attack_hold > 63 ||
          (f.buffer_action_id != -1 && !valid_action_id(f.buffer_action_id)) ||
          (f.reserve_action_id != -1 && !valid_action_id(f.reserve_action_id)) || f.facing_flipped > 1)
        return set_err(h, FS_E_INVALID, "fs_set_state: arena %d fighter %d out of representable range", i, k);
    }
    if (s.recording_count < 0 || s.recording_count > 18000)
      return set_err(h, FS_E_INVALID, "fs_set_state: arena %d recording_count out of range", i);
    if (!valid_bot(s.move_plan, s.move_index, s.attack_plan, s.attack_index, s.prev_opponent_action) ||
        !valid_bot(s.p1_move_plan, s.p1_move_index, s.p1_attack_plan, s.p1_attack_index,
                   s.p1_prev_opponent_action) ||
        s.bot_ready[0] > 1 || s.bot_ready[1] > 1 || s.bot_input[0] > 7 || s.bot_input[1] > 7 || s.p2_bot > 1)
      return set_err(h, FS_E_INVALID, "fs_set_state: arena %d bot state out of range", i);
    // a bot-created P2 is the bot for good and is Reset at every Intro (always ready); an idle P2
    // has no bot
    if ((h->cfg.p2_mode == FS_P2_BOT && (!s.p2_bot || !s.bot_ready[1])) ||
        (h->cfg.p2_mode == FS_P2_NOOP && s.p2_bot))
      return set_err(h, FS_E_INVALID, "fs_set_state: arena %d p2_bot / bot_ready do not fit the handle's P2 mode", i);
  }
  int rc;
  if ((rc = use_device(h))) return rc;
  fs_arena_state* d = nullptr;
  HIP_TRY(h, hipMalloc(&d, sizeof(fs_arena_state) * (size_t)h->n));
  hipError_t e = hipMemcpyAsync(d, host_in, sizeof(fs_arena_state) * (size_t)h->n, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = fsk::launch_set_state(h->st, d, h->n, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return set_err(h, FS_E_DEVICE, "fs_set_state: %s", hipGetErrorString(e));
  for (int i = 0; i < h->n; i++) set_p2bot_mirror(h, (size_t)i, host_in[i].p2_bot);
  // every arena was replaced: the general-geometry tick is needed iff a loaded fighter is off the
  // ground or faces the other way.  y is tested by its bits: a -0.0 moves no box, but the pushes
  // keep it (-0.0 + -0.0) and the round start writes +0.0 (SetupBattleStart, F:120-135), and only
  // the general-geometry tick carries y through a step (the standard one never writes it back)
  bool geom = false;
  for (int i = 0; i < h->n && !geom; i++)
    for (int k = 0; k < 2; k++)
      geom = geom || std::signbit(host_in[i].f[k].position_y) || host_in[i].f[k].position_y != 0.0f ||
             host_in[i].f[k].facing_flipped;
  h->geom = geom;
  return FS_OK;
}

FS_API int fs_sync(fs_handle h) {
  if (!h) return FS_E_INVALID;
  int rc;
  if ((rc = use_device(h))) return rc;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return FS_OK;
}

// Pinned, device-mapped host memory for callers without a device-memory library of their own (the
// torch-free Python surface binds its host outputs here): zero-filled, with its device address.
FS_API int fs_host_alloc(int device, size_t bytes, void** host, void** dev) {
  if (!host || !dev || !bytes) return set_err(nullptr, FS_E_INVALID, "fs_host_alloc: bytes > 0 and both pointers required");
  *host = *dev = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return set_err(nullptr, FS_E_DEVICE, "fs_host_alloc: hipSetDevice(%d): %s", device, hipGetErrorString(e));
  void* p = nullptr;
  e = hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable);
  if (e != hipSuccess) return set_err(nullptr, FS_E_OOM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
  memset(p, 0, bytes);
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, p, 0);
  if (e != hipSuccess || !d) {
    (void)hipHostFree(p);
    return set_err(nullptr, FS_E_DEVICE, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
  }
  *host = p;
  *dev = d;
  return FS_OK;
}

FS_API int fs_host_free(void* host) {
  if (!host) return FS_OK;
  hipError_t e = hipHostFree(host);
  return e == hipSuccess ? FS_OK : set_err(nullptr, FS_E_DEVICE, "hipHostFree: %s", hipGetErrorString(e));
}

// A synchronous copy between any two addresses the runtime knows (device, pinned host or pageable
// host; hipMemcpyDefault), for the same callers.
FS_API int fs_memcpy(void* dst, const void* src, size_t bytes) {
  if (!bytes) return FS_OK;
  if (!dst || !src) return set_err(nullptr, FS_E_INVALID, "fs_memcpy: null pointer");
  hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyDefault);
  return e == hipSuccess ? FS_OK : set_err(nullptr, FS_E_DEVICE, "fs_memcpy: %s", hipGetErrorString(e));
}

FS_API void* fs_stream(fs_handle h) { return h ? (void*)h->stream : nullptr; }
FS_API int fs_set_stream(fs_handle h, void* stream) {
  if (!h) return FS_E_INVALID;
  int rc;
  if ((rc = use_device(h))) return rc;
  hipStream_t next = stream == FS_STREAM_OWN ? h->own_stream : (hipStream_t)stream;
  if (next == h->stream) return FS_OK;
  // order the new stream after everything already issued on the old one
  HIP_TRY(h, hipEventRecord(h->staging_free, h->stream));
  HIP_TRY(h, hipStreamWaitEvent(next, h->staging_free, 0));
  h->stream = next;
  HIP_TRY(h, hipEventRecord(h->staging_free, h->stream));
  return FS_OK;
}

FS_API const char* fs_step_kernel(fs_handle h, int n_steps, int flags) {
  if (!h || n_steps <= 0 || (flags & ~(FS_KERNEL_HASHED | FS_KERNEL_POLICY | FS_KERNEL_PACKED))) return nullptr;
  return fsk::step_kernel_name((flags & FS_KERNEL_POLICY) != 0, (flags & FS_KERNEL_HASHED) != 0, n_steps, h->n,
                               h->cfg.float_mode, variant(h), h->geom, (flags & FS_KERNEL_PACKED) != 0,
                               h->cfg.autoreset_mode);
}

FS_API int fs_num_envs(fs_handle h) { return h ? h->n : 0; }
FS_API uint64_t fs_steps_taken(fs_handle h) { return h ? h->steps : 0; }

FS_API void fs_destroy(fs_handle h) {
  if (!h) return;
  if (hipSetDevice(h->device) == hipSuccess && h->stream) (void)hipStreamSynchronize(h->stream);
  free_all(h);
  delete h;
}

FS_API const char* fs_last_error(fs_handle h) { return h ? h->err.c_str() : g_create_error.c_str(); }

// ---------------------------------------------------------------------------
// host-side conversion of a step's outputs (fs_host_convert)
// ---------------------------------------------------------------------------
namespace {
// A fixed set of host worker threads, created on first use.  The pool object is never destroyed
// (its workers sleep on a condition variable until the process exits), and a forked child gets
// a fresh pool: the parent's workers do not exist there.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* pool = nullptr;
    static pid_t owner = 0;
    static std::mutex make;
    std::lock_guard<std::mutex> g(make);
    if (!pool || owner != getpid()) {
      pool = new HostPool();  // (a pool inherited through fork is abandoned, not destroyed)
      owner = getpid();
    }
    return *pool;
  }
  // fn(part, parts) for part = 0 .. parts - 1, part 0 on the calling thread; returns when all ran
  void run(int parts, const std::function<void(int, int)>& fn) {
    if (parts <= 1) {
      fn(0, 1);
      return;
    }
    std::lock_guard<std::mutex> serial(run_m_);  // one job at a time
    {
      std::lock_guard<std::mutex> g(m_);
      while ((int)workers_.size() < parts - 1) {
        const int id = (int)workers_.size();
        workers_.push_back(new std::thread([this, id] { loop(id); }));
      }
      fn_ = &fn;
      parts_ = parts;
      left_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0, parts);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int id) {  // worker id runs part id + 1 of the jobs that have that many parts
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return gen_ != seen; });
      seen = gen_;
      if (id + 1 >= parts_) continue;
      const std::function<void(int, int)>* fn = fn_;
      const int parts = parts_;
      g.unlock();
      (*fn)(id + 1, parts);
      g.lock();
      if (--left_ == 0) done_.notify_one();
    }
  }
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_;
  std::vector<std::thread*> workers_;
  const std::function<void(int, int)>* fn_ = nullptr;
  int parts_ = 0, left_ = 0;
  uint64_t gen_ = 0;
};
}  // namespace

static int host_convert_check(const fs_outputs* src, int64_t n_src, const int64_t* rows, int64_t n,
                              const fs_host_arrays* dst) {
  if (!src || !dst || n < 0 || n_src < 0)
    return set_err(nullptr, FS_E_INVALID, "fs_host_convert: src, dst, n >= 0 and n_src >= 0 required");
  if (!rows && n > n_src) return set_err(nullptr, FS_E_INVALID, "fs_host_convert: n exceeds the source's n_src rows");
  if (rows)  // every source row the conversion will read, checked before any thread starts
    for (int64_t i = 0; i < n; ++i)
      if (rows[i] < 0 || rows[i] >= n_src)
        return set_err(nullptr, FS_E_INVALID, "fs_host_convert: rows[i] outside [0, n_src)");
  const fs_outputs& S = *src;
  const fs_host_arrays& D = *dst;
  if ((D.guard || D.info_guard) && !S.guard) return set_err(nullptr, FS_E_INVALID, "fs_host_convert: no guard source");
  if ((D.move || D.info_move) && !S.move) return set_err(nullptr, FS_E_INVALID, "fs_host_convert: no move source");
  if ((D.move_frame || D.info_move_frame) && !S.move_frame)
    return set_err(nullptr, FS_E_INVALID, "fs_host_convert: no move_frame source");
  if ((D.position || D.info_position) && !S.position)
    return set_err(nullptr, FS_E_INVALID, "fs_host_convert: no position source");
  if ((D.frame && !S.frame) || ((D.p1_action || D.p2_action) && !S.action) ||
      ((D.p1_hitstun || D.p2_hitstun) && !S.hitstun) || (D.reward && !S.reward) ||
      (D.terminated && !S.terminated) || (D.truncated && !S.truncated))
    return set_err(nullptr, FS_E_INVALID, "fs_host_convert: a destination without its source");
  return FS_OK;
}

// the conversion proper (arguments checked), on `threads` of the host pool
static void host_convert_run(const fs_outputs S, const fs_host_arrays D, const int64_t* rows, int64_t n, int threads) {
  // below ~8k rows the threads' wake-up costs more than the conversion
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::max(threads, 1), n / 8192 + 1, 64}));
  HostPool::get().run(parts, [&](int part, int np) {
    const int64_t lo = n * part / np, hi = n * (part + 1) / np;
    // field by field over this part's rows (contiguous loops the compiler vectorizes); row r of
    // the source is rows[i] or i
    auto pairs = [&](auto* d, const auto* sp) {  // [N][2] -> [n][2]
      if (!d) return;
      if (!rows) {
        for (int64_t j = 2 * lo; j < 2 * hi; ++j) d[j] = sp[j];
      } else {
        for (int64_t i = lo; i < hi; ++i) {
          d[2 * i] = sp[2 * rows[i]];
          d[2 * i + 1] = sp[2 * rows[i] + 1];
        }
      }
    };
    auto single = [&](auto* d, const auto* sp, int stride, int k) {  // column k of [N][stride] -> [n]
      if (!d) return;
      if (!rows) {
        for (int64_t i = lo; i < hi; ++i) d[i] = sp[stride * i + k];
      } else {
        for (int64_t i = lo; i < hi; ++i) d[i] = sp[stride * rows[i] + k];
      }
    };
    pairs(D.guard, S.guard);
    pairs(D.info_guard, S.guard);
    pairs(D.move, S.move);
    pairs(D.info_move, S.move);
    pairs(D.move_frame, S.move_frame);
    pairs(D.info_move_frame, S.move_frame);
    pairs(D.position, S.position);
    pairs(D.info_position, S.position);
    single(D.frame, S.frame, 1, 0);
    single(D.p1_hitstun, S.hitstun, 2, 0);
    single(D.p2_hitstun, S.hitstun, 2, 1);
    single(D.reward, S.reward, 1, 0);
    for (int k = 0; k < 2; ++k) {
      uint8_t* act = k == 0 ? D.p1_action : D.p2_action;
      if (!act) continue;
      for (int64_t i = lo; i < hi; ++i) {
        const uint8_t a = S.action[2 * (rows ? rows[i] : i) + k];  // Left = 1, Right = 2, Attack = 4 (state.py:26-36)
        act[3 * i] = a & 1;
        act[3 * i + 1] = (a >> 1) & 1;
        act[3 * i + 2] = (a >> 2) & 1;
      }
    }
    for (int k = 0; k < 2; ++k) {
      uint8_t* d = k == 0 ? D.terminated : D.truncated;
      const uint8_t* sp = k == 0 ? S.terminated : S.truncated;
      if (!d) continue;
      for (int64_t i = lo; i < hi; ++i) d[i] = sp[rows ? rows[i] : i] != 0;
    }
  });
}

FS_API int fs_host_convert(const fs_outputs* src, int64_t n_src, const int64_t* rows, int64_t n,
                           const fs_host_arrays* dst, int threads) {
  const int rc = host_convert_check(src, n_src, rows, n, dst);
  if (rc) return rc;
  host_convert_run(*src, *dst, rows, n, threads);
  return FS_OK;
}

// fs_host_convert_start / _wait: one conversion at a time runs on a runner thread of its own (which
// drives the host pool as fs_host_convert's caller would), while the caller goes on with other work;
// a start while another thread's conversion is in flight waits for it first.
class AsyncConvert {
 public:
  static AsyncConvert& get() {
    static AsyncConvert* a = nullptr;
    static pid_t owner = 0;
    static std::mutex make;
    std::lock_guard<std::mutex> g(make);
    if (!a || owner != getpid()) {
      a = new AsyncConvert();  // (one inherited through fork is abandoned, as the pool)
      owner = getpid();
    }
    return *a;
  }
  void start(std::function<void()> job) {  // (after the conversion in flight, another thread's, ends)
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return !busy_; });
    if (!runner_) runner_ = new std::thread([this] { loop(); });
    job_ = std::move(job);
    busy_ = true;
    cv_.notify_one();
  }
  void wait() {  // until no conversion is in flight
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return !busy_; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [this] { return (bool)job_; });
      std::function<void()> job = std::move(job_);
      job_ = nullptr;
      g.unlock();
      job();
      g.lock();
      busy_ = false;
      done_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::thread* runner_ = nullptr;
  std::function<void()> job_;
  bool busy_ = false;
};

FS_API int fs_host_convert_start(const fs_outputs* src, int64_t n_src, const int64_t* rows, int64_t n,
                                 const fs_host_arrays* dst, int threads) {
  const int rc = host_convert_check(src, n_src, rows, n, dst);
  if (rc) return rc;
  const fs_outputs S = *src;
  const fs_host_arrays D = *dst;
  AsyncConvert::get().start([S, D, rows, n, threads] { host_convert_run(S, D, rows, n, threads); });
  return FS_OK;
}

FS_API int fs_host_convert_wait(void) {
  AsyncConvert::get().wait();
  return FS_OK;
}
