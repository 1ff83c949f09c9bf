// Back-to-back launch floor on one stream (measurement tool, not shipped):
// what a one-launch-per-step design pays before any work.  Per case: 2000 launches of a grid of
// 512 x 256 threads (k_step's grid at 65 536 arenas) between two events, after a warm-up.
//   empty   : the kernel returns at once
//   kernarg : reads its kernel arguments (one s_load) and stores one dword per thread
//   touch   : one dependent global load per thread (a 512 KB buffer), then one store per thread
//   touch3  : three dependent loads per thread, then one store (the tick's table-chain shape)
//   store_nt / load_only / store_1block: where the extra microseconds of a storing kernel come from
//   hbm136  : 144 B moved per arena, read and written (k_step moves 136), no compute
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor/launch_floor tools/launch_floor/floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_kernarg(unsigned* out, unsigned v) { out[blockIdx.x * blockDim.x + threadIdx.x] = v; }
__global__ void k_store_nt(unsigned* out, unsigned v) {
  __builtin_nontemporal_store(v, out + blockIdx.x * blockDim.x + threadIdx.x);
}
__global__ void k_load_only(const unsigned* in, unsigned* out) {  // stores only if the value is odd (never)
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned x = in[i];
  if (x & 1u) out[i] = x;
}
__global__ void k_touch(const unsigned* in, unsigned* out, int dep) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned x = i & 131071u;
  for (int d = 0; d < dep; d++) x = in[x] & 131071u;
  out[i] = x;
}
// 65 536 arenas x 2 lanes: each lane reads and writes 36 B (9 dwords): 9.4 MB a launch, k_step's 9.2 MB
__global__ void k_hbm(const unsigned* in, unsigned* out) {
  const unsigned l = blockIdx.x * blockDim.x + threadIdx.x, n = gridDim.x * blockDim.x;
  unsigned v[9];
#pragma unroll
  for (int j = 0; j < 9; j++) v[j] = in[j * n + l];
#pragma unroll
  for (int j = 0; j < 9; j++) out[j * n + l] = v[j] + 1;
}

template <class F>
static void timed(const char* name, F launch, bool last = false) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 200; i++) launch();
  (void)hipDeviceSynchronize();
  const int n = 2000;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < n; i++) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf(" \"%s\": %.3f%s\n", name, 1e3 * ms / n, last ? "" : ",");
}

int main() {
  const dim3 g(512), b(256);
  unsigned *in, *out;
  (void)hipMalloc(&in, 17u * 131072u * 4u);
  (void)hipMalloc(&out, 17u * 131072u * 4u);
  (void)hipMemset(in, 0, 17u * 131072u * 4u);
  printf("{\"grid\": [512, 256], \"us_per_launch\": {\n");
  timed("empty", [&] { hipLaunchKernelGGL(k_empty, g, b, 0, 0); });
  timed("kernarg", [&] { hipLaunchKernelGGL(k_kernarg, g, b, 0, 0, out, 7u); });
  timed("touch", [&] { hipLaunchKernelGGL(k_touch, g, b, 0, 0, in, out, 1); });
  timed("touch3", [&] { hipLaunchKernelGGL(k_touch, g, b, 0, 0, in, out, 3); });
  timed("hbm136", [&] { hipLaunchKernelGGL(k_hbm, g, b, 0, 0, in, out); });
  timed("store_nt", [&] { hipLaunchKernelGGL(k_store_nt, g, b, 0, 0, out, 7u); });
  timed("load_only", [&] { hipLaunchKernelGGL(k_load_only, g, b, 0, 0, in, out); });
  timed("store_1block", [&] { hipLaunchKernelGGL(k_kernarg, dim3(1), dim3(64), 0, 0, out, 7u); });
  timed("empty_1block", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0); }, true);
  printf("}}\n");
  return 0;
}
