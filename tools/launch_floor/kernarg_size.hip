// Does the size of a launch's kernel arguments cost time?  (measurement tool, not shipped; VERDICT
// r03 item 4: the step kernels pass a 352-B StepParams by value.)  Per size S in {16, 64, 128,
// 256, 352, 512} B: a kernel over k_step's grid (512 x 256 threads) whose argument is an S-byte
// struct; every thread reads the struct's last dword and stores it.  Timed two ways:
//   region : host wall clock of hipStreamSynchronize; launch; hipStreamSynchronize (median of 400),
//            the shape of one bench.py timed region;
//   b2b    : the launch-to-launch period of 2000 back-to-back launches between two events;
//   host   : host time of the launch call alone (median of 400, the stream drained before each).
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor/kernarg_size tools/launch_floor/kernarg_size.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

template <int S>
struct Args {
  unsigned w[S / 4];
};

template <int S>
__global__ void k_args(Args<S> a, unsigned* out) {
  out[blockIdx.x * blockDim.x + threadIdx.x] = a.w[S / 4 - 1];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int S>
static void run(unsigned* out, hipStream_t s) {
  Args<S> a{};
  for (int i = 0; i < S / 4; i++) a.w[i] = i;
  const dim3 g(512), b(256);
  for (int i = 0; i < 50; i++) hipLaunchKernelGGL(k_args<S>, g, b, 0, s, a, out);
  hipStreamSynchronize(s);
  std::vector<double> region, host;
  for (int i = 0; i < 400; i++) {
    hipStreamSynchronize(s);
    const double t0 = now_us();
    hipLaunchKernelGGL(k_args<S>, g, b, 0, s, a, out);
    const double t1 = now_us();
    hipStreamSynchronize(s);
    const double t2 = now_us();
    region.push_back(t2 - t0);
    host.push_back(t1 - t0);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int i = 0; i < 2000; i++) hipLaunchKernelGGL(k_args<S>, g, b, 0, s, a, out);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::sort(region.begin(), region.end());
  std::sort(host.begin(), host.end());
  printf("{\"kernarg_bytes\": %d, \"region_us\": %.2f, \"host_launch_us\": %.2f, \"b2b_us\": %.3f}\n", S,
         region[region.size() / 2], host[host.size() / 2], 1e3 * ms / 2000);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  unsigned* out;
  hipMalloc(&out, 512 * 256 * sizeof(unsigned));
  hipStream_t s;
  hipStreamCreate(&s);
  for (int rep = 0; rep < 2; rep++) {
    run<16>(out, s);
    run<64>(out, s);
    run<128>(out, s);
    run<256>(out, s);
    run<352>(out, s);
    run<512>(out, s);
  }
  hipFree(out);
  return 0;
}
