// What a kernel's output stores cost at the end of the launch, by cache policy (measurement tool,
// not shipped).  A storing kernel costs ~1.5 us more per back-to-back launch than an empty one
// (floor.hip: the end-of-kernel release writes dirty L2 lines back); does that depend on the
// store's cache policy and on how much was written?  Per case: 1000 back-to-back launches of
// 512 x 256 threads between two events, each thread storing `per` dwords (the C3 20-tick launch
// writes ~50 MB of outputs: per = 96), and the same for a sync-launch-sync region timed on the
// host (what bench.py's driver-shape region pays per launch).
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor/store_policy tools/launch_floor/store_policy.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int POL>
__device__ __forceinline__ void st(unsigned* p, unsigned v) {
  if constexpr (POL == 0) *p = v;
  else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
  else if constexpr (POL == 2) asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 3) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 4) asm volatile("global_store_dword %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

template <int POL>
__global__ __launch_bounds__(256) void k_store(unsigned* out, int per, unsigned v) {
  const unsigned n = gridDim.x * blockDim.x, i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int j = 0; j < per; j++) st<POL>(out + (size_t)j * n + i, v + j);
}

template <int POL>
static void run(const char* name, unsigned* out, int per, bool last) {
  const dim3 g(512), b(256);
  for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_store<POL>, g, b, 0, 0, out, per, 7u);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int n = 1000;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_store<POL>, g, b, 0, 0, out, per, (unsigned)i);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // sync - launch - sync regions, host clock (median of 201)
  double t[201];
  for (int i = 0; i < 201; i++) {
    (void)hipDeviceSynchronize();
    const auto a = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_store<POL>, g, b, 0, 0, out, per, (unsigned)i);
    (void)hipDeviceSynchronize();
    t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  }
  for (int i = 1; i < 201; i++)
    for (int j = i; j > 0 && t[j] < t[j - 1]; j--) {
      const double x = t[j]; t[j] = t[j - 1]; t[j - 1] = x;
    }
  printf("  {\"policy\": \"%s\", \"dwords_per_thread\": %d, \"mb\": %.1f, \"b2b_us\": %.3f, \"region_us\": %.3f}%s\n", name,
         per, per * 512.0 * 256 * 4 / 1e6, 1e3 * ms / n, t[100], last ? "" : ",");
}

int main() {
  unsigned* out = nullptr;
  if (hipMalloc(&out, 96u * 512u * 256u * 4u) != hipSuccess || !out) return 1;
  printf("{\"grid\": [512, 256], \"cases\": [\n");
  for (int per : {1, 96}) {
    run<0>("default", out, per, false);
    run<1>("nt", out, per, false);
    run<2>("sc0 sc1", out, per, false);
    run<3>("sc1", out, per, false);
    run<4>("sc0", out, per, false);
    run<5>("sc0 sc1 nt", out, per, per == 96);
  }
  printf("]}\n");
  return 0;
}
