// Host-side share of a synchronize-launch-synchronize region (measurement tool, not shipped):
// the same one-store-per-thread kernel of C3's grid (512 x 256), the region timed on the host
// (median of 401) under each device scheduling flag (set before the context exists, so one
// process per flag: `sync_modes FLAG`) and with device- vs stream-synchronize.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor/sync_modes tools/launch_floor/sync_modes.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_store(unsigned* out, unsigned v) { out[blockIdx.x * blockDim.x + threadIdx.x] = v; }

static double median_region(unsigned* out, hipStream_t s, bool stream_sync, bool empty) {
  std::vector<double> t(401);
  for (int i = 0; i < 401; i++) {
    if (stream_sync) (void)hipStreamSynchronize(s);
    else (void)hipDeviceSynchronize();
    const auto a = std::chrono::steady_clock::now();
    if (!empty) hipLaunchKernelGGL(k_store, dim3(512), dim3(256), 0, s, out, (unsigned)i);
    if (stream_sync) (void)hipStreamSynchronize(s);
    else (void)hipDeviceSynchronize();
    t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  }
  std::sort(t.begin(), t.end());
  return t[200];
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "auto";
  unsigned flag = hipDeviceScheduleAuto;
  if (!strcmp(mode, "spin")) flag = hipDeviceScheduleSpin;
  else if (!strcmp(mode, "yield")) flag = hipDeviceScheduleYield;
  else if (!strcmp(mode, "blocking")) flag = hipDeviceScheduleBlockingSync;
  if (hipSetDeviceFlags(flag) != hipSuccess) {
    printf("{\"mode\": \"%s\", \"error\": \"hipSetDeviceFlags\"}\n", mode);
    return 0;
  }
  unsigned* out = nullptr;
  if (hipMalloc(&out, 512 * 256 * 4) != hipSuccess || !out) return 1;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  for (int i = 0; i < 200; i++) hipLaunchKernelGGL(k_store, dim3(512), dim3(256), 0, s, out, 1u);
  (void)hipDeviceSynchronize();
  const double dev_empty = median_region(out, s, false, true), dev = median_region(out, s, false, false);
  const double str_empty = median_region(out, s, true, true), str = median_region(out, s, true, false);
  printf("{\"mode\": \"%s\", \"device_sync_region_us\": %.3f, \"device_sync_empty_us\": %.3f, "
         "\"stream_sync_region_us\": %.3f, \"stream_sync_empty_us\": %.3f}\n", mode, dev, dev_empty, str, str_empty);
  return 0;
}
