// bench_native -- the C-ABI driven from C++ with no Python in the loop ("the
// C++ benchmark driver").  The same C3 workload as bench.py: N arenas (default 65 536), P2 a
// remote actor, splitmix64 self-play actions made resident in HBM by fs_hash_actions, every
// tick's outputs kept in a [ticks][N] trajectory.  Per launch shape (ticks per fs_step_n) it
// times R regions of exactly one launch each, bracketed by hipDeviceSynchronize on the host
// clock (bench.py's region with ctypes / torch out of it), and the same launches back to back
// with HIP events on the handle's stream; then fs_step (one tick per launch) both ways.
// Prints one JSON object.
//   make -C tools/bench_native            (links footsies_gym_amd/libfootsies.so)
//   tools/bench_native/bench_native [N] [regions]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/footsies.h"

#define FS_CHECK(h, x)                                                            \
  do {                                                                            \
    const int rc_ = (x);                                                          \
    if (rc_ != FS_OK) {                                                           \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_, fs_last_error(h)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)
#define HIP_CHECK(x)                                                                        \
  do {                                                                                      \
    const hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

struct Traj {
  fs_outputs o{};
  std::vector<void*> bufs;
  void alloc(size_t rows, size_t n) {
    auto dev = [&](size_t bytes) {
      void* p = nullptr;
      HIP_CHECK(hipMalloc(&p, bytes));
      HIP_CHECK(hipMemset(p, 0, bytes));
      bufs.push_back(p);
      return p;
    };
    const size_t r = rows * n;
    o.guard = (uint8_t*)dev(2 * r);
    o.move = (uint8_t*)dev(2 * r);
    o.move_frame = (float*)dev(8 * r);
    o.position = (float*)dev(8 * r);
    o.reward = (double*)dev(8 * r);
    o.terminated = (uint8_t*)dev(r);
    o.truncated = (uint8_t*)dev(r);
    o.frame = (int32_t*)dev(4 * r);
    o.action = (uint8_t*)dev(2 * r);
    o.hitstun = (uint8_t*)dev(2 * r);
    o.final_guard = (uint8_t*)dev(2 * r);
    o.final_move = (uint8_t*)dev(2 * r);
    o.final_move_frame = (float*)dev(8 * r);
    o.final_position = (float*)dev(8 * r);
    o.final_frame = (int32_t*)dev(4 * r);
    o.final_action = (uint8_t*)dev(2 * r);
    o.final_hitstun = (uint8_t*)dev(2 * r);
  }
  ~Traj() {
    for (void* p : bufs) (void)hipFree(p);
  }
};

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 65536;
  const int R = argc > 2 ? atoi(argv[2]) : 21;
  if (N <= 0 || R <= 0) return 1;
  fs_config cfg{};
  cfg.num_envs = N;
  cfg.p2_mode = FS_P2_EXTERNAL;
  cfg.dense_reward = 1;
  cfg.float_mode = FS_FLOAT_STRICT32;
  cfg.autoreset_mode = FS_AUTORESET_SAME_STEP;
  fs_handle h = nullptr;
  FS_CHECK(nullptr, fs_create(&cfg, &h));
  const int shapes[] = {1000, 20};
  const int max_ticks = 1000, rows = 2 * R * max_ticks + 200;  // fresh action rows per launch
  uint8_t *p1 = nullptr, *p2 = nullptr;
  HIP_CHECK(hipMalloc(&p1, (size_t)rows * N));
  HIP_CHECK(hipMalloc(&p2, (size_t)rows * N));
  FS_CHECK(h, fs_hash_actions(h, rows, 0x5EED, 0, p1, p2));
  Traj traj;
  traj.alloc(max_ticks, N);
  FS_CHECK(h, fs_sync(h));
  hipStream_t s = (hipStream_t)fs_stream(h);
  printf("{\"envs\": %d, \"regions\": %d, \"shapes\": [", N, R);
  size_t row = 0;
  auto next_rows = [&](int ticks) {
    if (row + ticks > (size_t)rows) row = 0;
    const size_t r0 = row;
    row += ticks;
    return r0;
  };
  for (int si = 0; si < 2; si++) {
    const int T = shapes[si];
    // warm-up
    for (int w = 0; w < 3; w++) {
      const size_t r0 = next_rows(T);
      FS_CHECK(h, fs_step_n(h, T, p1 + r0 * N, p2 + r0 * N, 0, &traj.o));
    }
    HIP_CHECK(hipDeviceSynchronize());
    std::vector<double> region(R), host_call(R);
    for (int r = 0; r < R; r++) {
      const size_t r0 = next_rows(T);
      HIP_CHECK(hipDeviceSynchronize());
      const auto a = std::chrono::steady_clock::now();
      FS_CHECK(h, fs_step_n(h, T, p1 + r0 * N, p2 + r0 * N, 0, &traj.o));
      const auto b = std::chrono::steady_clock::now();
      HIP_CHECK(hipDeviceSynchronize());
      const auto c = std::chrono::steady_clock::now();
      region[r] = std::chrono::duration<double, std::micro>(c - a).count();
      host_call[r] = std::chrono::duration<double, std::micro>(b - a).count();
    }
    // back to back, HIP events on the handle's stream
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    const int L = T >= 1000 ? 5 : 200;
    HIP_CHECK(hipEventRecord(e0, s));
    for (int l = 0; l < L; l++) {
      const size_t r0 = next_rows(T);
      FS_CHECK(h, fs_step_n(h, T, p1 + r0 * N, p2 + r0 * N, 0, &traj.o));
    }
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double b2b = 1e3 * ms / L, reg = median(region);
    printf("%s{\"ticks_per_launch\": %d, \"region_us\": %.2f, \"region_env_steps_per_s\": %.4e, "
           "\"host_call_us\": %.2f, \"back_to_back_us\": %.2f, \"back_to_back_env_steps_per_s\": %.4e}",
           si ? ", " : "", T, reg, (double)N * T / (reg * 1e-6), median(host_call), b2b,
           (double)N * T / (b2b * 1e-6));
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
  }
  // fs_step: one tick per launch
  {
    const int K = 300;
    for (int k = 0; k < 20; k++) FS_CHECK(h, fs_step(h, p1 + (size_t)k * N, p2 + (size_t)k * N, FS_ACT_DEVICE));
    HIP_CHECK(hipDeviceSynchronize());
    const auto a = std::chrono::steady_clock::now();
    for (int k = 0; k < K; k++) FS_CHECK(h, fs_step(h, p1 + (size_t)k * N, p2 + (size_t)k * N, FS_ACT_DEVICE));
    HIP_CHECK(hipDeviceSynchronize());
    const double per = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count() / K;
    std::vector<double> reg(R);
    for (int r = 0; r < R; r++) {
      HIP_CHECK(hipDeviceSynchronize());
      const auto b = std::chrono::steady_clock::now();
      FS_CHECK(h, fs_step(h, p1 + (size_t)r * N, p2 + (size_t)r * N, FS_ACT_DEVICE));
      HIP_CHECK(hipDeviceSynchronize());
      reg[r] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - b).count();
    }
    printf("], \"fs_step\": {\"back_to_back_us\": %.2f, \"env_steps_per_s\": %.4e, \"region_us\": %.2f}}\n", per,
           (double)N / (per * 1e-6), median(reg));
  }
  HIP_CHECK(hipFree(p1));
  HIP_CHECK(hipFree(p2));
  fs_destroy(h);
  return 0;
}
